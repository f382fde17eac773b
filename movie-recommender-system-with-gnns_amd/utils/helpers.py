"""Triplet sampling for BPR training — the reference's utils/helpers.py:64-102 API.

``get_triplets_indices(edge_index, num_users, num_items, device)`` returns
(users, positive items, negative items) for one batch edge list:
  * users = sources that are users, positives = targets that are items (shifted to item ids).
    Because the graph is bipartite and symmetrised, the k-th user->item edge gives both the k-th
    user and the k-th positive;
  * negatives are uniform over all items with no filtering of positives, drawn with
    ``torch.randint`` on ``device`` from the global generator, so a fixed torch seed reproduces
    the reference's draws exactly (Q9).
The reference's unused helpers (cantor_hash_pair / get_user_items / is_in_feasible,
utils/helpers.py:11-62, no call sites) are not carried over.
"""
from typing import Tuple

import torch

torch.manual_seed(0)  # import-time seeding, as reference utils/helpers.py:5-9
torch.cuda.manual_seed(0)
torch.cuda.manual_seed_all(0)


def sample_negative(pos_idx: torch.Tensor, num_items: int, device) -> torch.Tensor:
    """One uniform random item per positive (reference utils/helpers.py:64-82)."""
    return torch.randint(0, num_items, (pos_idx.shape[0],), device=device)


# the function above as defined here, whatever a caller later patches sample_negative to
# (lgcn_amd.harness draws in place only while the two are the same object)
REFERENCE_SAMPLE_NEGATIVE = sample_negative


def get_triplets_indices(edge_index: torch.Tensor, num_users: int, num_items: int,
                         device) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(user ids, positive item ids, negative item ids) of a batch (reference utils/helpers.py:84-102)."""
    src, dst = edge_index[0], edge_index[1]
    users = src[src < num_users]
    positives = dst[dst >= num_users] - num_users
    negatives = sample_negative(positives, num_items, device)
    return users, positives, negatives
