"""LightGCN with the reference's API, propagating on MI355X HIP kernels.

Drop-in for reference models/light_gcn.py (class LightGCN, :13-64):
  * constructor ``LightGCN(num_users, num_items, num_layers=4, dim_h=64)`` (:14), two
    ``nn.Embedding`` tables initialised ``normal_(std=0.01)`` (:22-26);
  * ``forward(edge_index) -> (users [U,d], items [I,d])`` (:28-40), with the reference's
    layer-stack scaling ``1/(K+1) * mean(stack(embs))`` (:36);
  * ``get_embeddings`` (:42-64) returning raw layer-0 rows or ``(None, None)`` + UserWarning;
  * state_dict keys exactly ``user_embedding.weight`` / ``item_embedding.weight`` (Q12).
The K LGConv layers run as one autograd node on a cached device plan (lgcn_amd); the
per-layer ``convs`` list is kept (parameter-free) for API compatibility only.
There is no CPU path: forward raises unless the model and edge_index live on a ROCm device.
"""
import warnings

import torch
import torch.nn as nn

import lgcn_amd
from lgcn_amd.plan import PlanCache

# Same import-time seeding as the reference (models/light_gcn.py:7-11), so a model built right
# after import starts from the reference's initial weights.
torch.manual_seed(0)
torch.cuda.manual_seed(0)
torch.cuda.manual_seed_all(0)
torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False


class LightGCN(nn.Module):
    def __init__(self, num_users, num_items, num_layers=4, dim_h=64):
        super().__init__()
        self.num_users = num_users
        self.num_items = num_items
        self.num_layers = num_layers
        self.dim_h = dim_h

        self.user_embedding = nn.Embedding(num_embeddings=self.num_users, embedding_dim=dim_h)
        self.item_embedding = nn.Embedding(num_embeddings=self.num_items, embedding_dim=dim_h)
        self.convs = nn.ModuleList(lgcn_amd.LGConv() for _ in range(num_layers))
        nn.init.normal_(self.user_embedding.weight, std=0.01)
        nn.init.normal_(self.item_embedding.weight, std=0.01)
        self._plans = PlanCache()

    def plan_for(self, edge_index):
        """The cached propagation plan of an edge set (built on first use)."""
        return self._plans.get(edge_index, self.num_users + self.num_items, side_split=self.num_users)

    def forward(self, edge_index):
        plan = self.plan_for(edge_index)
        emb_final = lgcn_amd.lightgcn_propagate(self.user_embedding.weight, self.item_embedding.weight,
                                                plan, self.num_layers)
        emb_users_final, emb_items_final = torch.split(emb_final, [self.num_users, self.num_items])
        return emb_users_final, emb_items_final

    def get_embeddings(self, user_indices=None, item_indices=None):
        """Raw (layer-0) rows, as reference models/light_gcn.py:42-64."""
        if user_indices is not None and item_indices is not None:
            return self.user_embedding.weight[user_indices], self.item_embedding.weight[item_indices]
        if user_indices is not None:
            return self.user_embedding.weight[user_indices], None
        if item_indices is not None:
            return None, self.item_embedding.weight[item_indices]
        warnings.warn("Both indices not provided", UserWarning)
        return None, None
