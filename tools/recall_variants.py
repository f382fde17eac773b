"""A/B timing of k_score_filter variants (built by tools/build_recall_variants.sh into
tools/_variants/): the full pass of the C3 eval shape (Q=1000 users, M=1.24M candidates, d=128).
python tools/recall_variants.py"""
import ctypes
import glob
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "movie-recommender-system-with-gnns_amd"))
from lgcn_amd import _ffi  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    Q, M, d, k = 1000, 1243124, 128, 100
    users = torch.randn(620000, d, device=dev)
    cand = torch.randn(M, d, device=dev)
    picked = torch.from_numpy(np.random.default_rng(0).choice(620000, Q, replace=False)).to(dev)
    libs = {"main": _ffi.load()}
    for p in sorted(glob.glob(os.path.join(ROOT, "tools", "_variants", "*.so"))):
        lib = ctypes.CDLL(p)
        for name, (args, res) in _ffi._SIGS.items():
            if hasattr(lib, name):
                f = getattr(lib, name)
                f.argtypes, f.restype = args, res
        libs[os.path.basename(p)[:-3]] = lib
    from lgcn_amd import recall

    hits_ref = recall.topk_hits(users, picked, cand[:M // 2], cand[M // 2:], k)
    ws = recall._WS
    s = _ffi.stream_of(dev)
    Qpad = ws.Qn.shape[0]
    for rep in range(3):
        for name, lib in libs.items():
            ws.lcnt.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(3):
                ws.lcnt.zero_()
                rc = lib.lgcn_score_filter(ws.Qn.data_ptr(), Qpad, Q, ws.Cn.data_ptr(), M, 1, 128, ws.thr.data_ptr(),
                                           ws.lkey.data_ptr(), ws.lidx.data_ptr(), ws.lcnt.data_ptr(), 16384, s)
                assert rc == 0
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 3
            print(f"{name:24s} {ms:7.3f} ms  {2 * 1024 * M * d / ms / 1e9:6.1f} TFLOP/s  max list {int(ws.lcnt.max())}",
                  flush=True)


if __name__ == "__main__":
    main()
