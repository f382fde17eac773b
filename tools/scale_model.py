"""The event model that prices a reduce-mode C2 grid's K-layer step from its pieces (shared by
tools/project_scale.py, which prices from one-GPU pieces and an assumed bus bandwidth, and
bench.py --gpus N, which prices the chosen grid from the same pieces and the collectives it just
timed on the node, and prints the projection beside the measured step).

A rank's step (reference models/light_gcn.py:32-36, one LGConv per layer, rows sharded):
  overlapped: P_k (the partial item pass over the rank's users) -> all_reduce_k on the collective
              stream; U_k (the user pass) waits for all_reduce_{k-1}; the last layer's collective is
              a reduce_scatter.
  fused:      pair_k = P_k and U_k in one launch, then all_reduce_k; pair_{k+1} waits for it.
"""
from __future__ import annotations

# bytes a collective moves per rank over its links, as a multiple of the buffer (ring algorithms):
# the "bus bandwidth" convention of rccl-tests / nccl-tests
BUS_FACTOR = {
    "all_reduce": lambda n: 2.0 * (n - 1) / n,
    "reduce_scatter": lambda n: (n - 1) / n,
    "all_gather": lambda n: (n - 1) / n,
    "all_to_all": lambda n: (n - 1) / n,
}


def bus_gbps(op: str, nbytes: int, n: int, ms: float) -> float:
    """bus bandwidth (GB/s) of one collective of `nbytes` (the full buffer) over n ranks in ms."""
    return BUS_FACTOR[op](n) * nbytes / (ms * 1e-3) / 1e9 if ms > 0 else float("nan")


def simulate(K, t_p, t_u, t_pair, t_ar, t_rs, fused):
    """ms per K-layer step of one rank (compute on one stream, the collectives serialised on
    another); the final stack mean (a few us) is ignored."""
    if fused:
        t, ar_done = 0.0, 0.0
        for k in range(1, K + 1):
            t = max(t, ar_done) + t_pair
            ar_done = t + (t_ar if k < K else t_rs)
        return ar_done
    t, comm, ar_done = 0.0, 0.0, {0: 0.0}
    for k in range(1, K + 1):
        t += t_p  # P_k needs U_{k-1}: the compute stream is in order
        comm = max(comm, t) + (t_ar if k < K else t_rs)
        ar_done[k] = comm
        t = max(t, ar_done[k - 1]) + t_u  # U_k reads the items reduced one layer earlier
    return max(t, ar_done[K])
