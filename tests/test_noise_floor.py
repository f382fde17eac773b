"""The oracle's own Recall noise floor at C1 size: the CPU oracle harness run a
second and third time with other valid summation orders (each LGConv's edges and each batch's
triplets permuted — the same arithmetic, another association), tests/c1_harness.py. The tables
move apart at the fp32 rounding level (asserted: they differ, and stay within the trajectory bar),
Recall@20 / @100 do not move at all (spread 0). tests/test_gpu_training.py::
test_recall_parity_c1_size holds the GPU path to max(1e-3 relative, 2 x this spread)."""
import numpy as np
import torch

import c1_harness as C
from parity import record_stats, trajectory_bar


def test_oracle_recall_noise_floor_c1():
    cpu = torch.device("cpu")
    data = C.c1_data()
    init = C.init_state()
    w0 = [init["user_embedding.weight"].numpy(), init["item_embedding.weight"].numpy()]
    m, gs, _ = C.train_c1(cpu, data=data, init=init)
    w_ref = C.tables(m)
    rec_ref = C.recall(w_ref, cpu, gs, data=data)
    spread = {20: 0.0, 100: 0.0}
    stats = {"recall_ref": rec_ref}
    for seed in (1, 2):
        m2, gs2, _ = C.train_c1(cpu, order_seed=seed, data=data, init=init)
        assert torch.equal(gs2, gs)  # the same negatives were drawn
        w = C.tables(m2)
        assert any(not torch.equal(a, b) for a, b in zip(w, w_ref))  # the order really changed the sums
        for t, name in enumerate(("user", "item")):
            stats[f"order{seed}.{name}"] = trajectory_bar(w[t].numpy(), w_ref[t].numpy(), w0[t],
                                                          np.ones(w0[t].shape, bool), 1e-3, C.EPOCHS * len(data[2]),
                                                          f"second order {seed} {name}", max_frac=1e-3, rtol=1e-3)
        rec = C.recall(w, cpu, gs, data=data)
        for k in (20, 100):
            spread[k] = max(spread[k], abs(rec[k] - rec_ref[k]))
        stats[f"order{seed}.recall"] = rec
    stats["spread"] = spread
    record_stats("oracle_noise_floor_c1", stats)
    print(f"oracle Recall@20/@100 {rec_ref[20]:.8f} / {rec_ref[100]:.8f}; spread over two other summation "
          f"orders {spread[20]:.2e} / {spread[100]:.2e}")
    assert spread[20] <= 2e-4 and spread[100] <= 2e-4, spread
