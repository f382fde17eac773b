"""The on-device content digest (lgcn_digest128, csrc/lgcn_plan.hip) behind lgcn_amd._cache's keys
for device tensors, and the harness paths it serves:

* the digest bitwise equal to its numpy restatement below, sensitive to one changed byte, a swap
  of two words, the length, and deterministic;
* a loader that collates NEW DEVICE edge_index tensors every epoch (the reference's PyG DataLoader
  on a GPU, data/dataset_handler.py:285) replays each batch's captured graph — bitwise the
  same-object run — with the digests prefetched one batch ahead;
* the row-lazy Adam's step-constant table grown at an epoch's start (sized loader) and mid-epoch
  (a loader without len()) — bitwise a run whose table never grows; the batch caches of a loader
  without len() grow with the batches it yields."""
import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _u(x):
    return np.uint64(x)


def _fmix64(k):
    with np.errstate(over="ignore"):
        k = k ^ (k >> _u(33))
        k = k * _u(0xFF51AFD7ED558CCD)
        k = k ^ (k >> _u(33))
        k = k * _u(0xC4CEB9FE1A85EC53)
        k = k ^ (k >> _u(33))
    return k


def digest_ref(buf: bytes) -> bytes:
    """numpy restatement of lgcn_digest128 (uint64 arithmetic wraps mod 2^64)."""
    n = len(buf)
    nw = n // 8
    words = np.frombuffer(buf[:nw * 8], dtype=np.uint64)
    if n % 8:
        words = np.concatenate([words, np.frombuffer(buf[nw * 8:] + b"\0" * (8 - n % 8), dtype=np.uint64)])
    i = np.arange(words.size, dtype=np.uint64)
    with np.errstate(over="ignore"):
        a = _fmix64(words ^ _fmix64(i * _u(0x9E3779B97F4A7C15) + _u(0x243F6A8885A308D3)))
        b = _fmix64(((words + _u(0x632BE59BD9B4E019)) * _u(0xD6E8FEB86659FD93)) ^ _fmix64(i + _u(0x8CB92BA72F3D8DD7)))
        sa, sb = _u(int(a.sum(dtype=np.uint64))), _u(int(b.sum(dtype=np.uint64)))
        o0 = _fmix64(np.array([sa ^ _u(n)], dtype=np.uint64))
        o1 = _fmix64(np.array([sb + _u(n) * _u(0x9E3779B97F4A7C15)], dtype=np.uint64))
    return np.concatenate([o0, o1]).tobytes()


def _dev_digest(t):
    from lgcn_amd import _cache

    return _cache._device_digest_start(t).result()


@pytest.mark.parametrize("shape,dtype", [((2, 20011), torch.int64), ((2, 1), torch.int64), ((0,), torch.int64),
                                         ((2, 3_000_000), torch.int64), ((7,), torch.uint8), ((13,), torch.int32),
                                         ((5, 33), torch.float32)])
def test_digest_matches_restatement(gpu, shape, dtype):
    g = torch.Generator().manual_seed(sum(shape) + 1)
    if dtype.is_floating_point:
        t = torch.randn(shape, generator=g).to(dtype)
    else:
        t = torch.randint(0, 200, shape, generator=g).to(dtype)
    want = digest_ref(t.numpy().tobytes())
    assert _dev_digest(t.to(gpu)) == want
    assert _dev_digest(t.to(gpu)) == want  # deterministic (another grid of partial sums, same value)


def test_digest_sensitivity(gpu):
    g = torch.Generator().manual_seed(3)
    ei = torch.randint(0, 100000, (2, 50000), generator=g)
    base = _dev_digest(ei.to(gpu))
    one = ei.clone()
    one[1, 777] += 1
    swap = ei.clone()
    swap[0, 10], swap[0, 11] = ei[0, 11].item(), ei[0, 10].item()
    assert ei[0, 10] != ei[0, 11]
    shorter = ei[:, :-1].contiguous()
    seen = {base}
    for t in (one, swap, shorter):
        d = _dev_digest(t.to(gpu))
        assert d not in seen
        seen.add(d)
    # a non-contiguous view digests its contiguous content
    assert _dev_digest(ei.to(gpu).t().contiguous().t()) == base
    # a byte view at an odd offset: the same bytes' digest (an aligned copy is hashed)
    raw = torch.arange(0, 37, dtype=torch.uint8)
    dev_raw = raw.to(gpu)
    assert _dev_digest(dev_raw[3:]) == digest_ref(raw[3:].numpy().tobytes())


class _B:
    def __init__(self, ei):
        self.edge_index = ei

    def to(self, device):
        return _B(self.edge_index.to(device))


class _FreshDevice:
    """Yields a new device edge_index (a clone) per batch every epoch."""

    def __init__(self, arrays, gpu):
        self.src = [torch.from_numpy(a).to(gpu) for a in arrays]

    def __len__(self):
        return len(self.src)

    def __iter__(self):
        for t in self.src:
            yield _B(t.clone())


def _run(gpu, U, I, init, loader, epochs, lr=1e-3):
    from lgcn_amd import harness
    from models.light_gcn import LightGCN
    from utils import train_test as TT

    m = LightGCN(U, I, num_layers=3, dim_h=64).to(gpu)
    with torch.no_grad():
        m.user_embedding.weight.copy_(init[0])
        m.item_embedding.weight.copy_(init[1])
    opt = torch.optim.Adam(m.parameters(), lr=lr)
    torch.manual_seed(41)
    losses = []
    for _ in range(epochs):
        losses.append(TT.train(m, opt, loader() if callable(loader) else loader, gpu))
        assert TT.LAST_TRAIN_PATH == "fused", TT.LAST_TRAIN_PATH
    st = [opt.state[p] for p in (m.user_embedding.weight, m.item_embedding.weight)]
    out = dict(losses=losses, w=[m.user_embedding.weight.detach().cpu().clone(), m.item_embedding.weight.detach().cpu().clone()],
               m=[s["exp_avg"].cpu().clone() for s in st], v=[s["exp_avg_sq"].cpu().clone() for s in st],
               step=[float(s["step"]) for s in st])
    return out, harness._FAST[opt]


def _golden():
    G = np.load(GOLDEN / "harness.npz")
    U, I = int(G["train_U"]), int(G["train_I"])
    init = (torch.from_numpy(G["train_init_user_w"]), torch.from_numpy(G["train_init_item_w"]))
    return U, I, init, [G[f"train_batch{p}"] for p in range(3)]


def _assert_same(a, b):
    assert a["losses"] == b["losses"], (a["losses"], b["losses"])
    assert a["step"] == b["step"]
    for k in ("w", "m", "v"):
        for x, y in zip(a[k], b[k]):
            assert torch.equal(x, y), k


def test_harness_fresh_device_tensors_replay_without_sync(gpu, tune):
    """New device tensors every epoch: each batch's state found by its prefetched device digest,
    bitwise the same-object run, one state and one captured graph per distinct batch."""
    from lgcn_amd import _cache

    tune(harness_fused=True)
    U, I, init, arrays = _golden()
    same = [_B(torch.from_numpy(a).to(gpu)) for a in arrays]
    ref, _ = _run(gpu, U, I, init, same, 4)
    calls = {"n": 0}
    orig = _cache._device_digest_start

    def counted(t):
        calls["n"] += 1
        return orig(t)

    _cache._device_digest_start = counted
    try:
        got, fast = _run(gpu, U, I, init, _FreshDevice(arrays, gpu), 4)
    finally:
        _cache._device_digest_start = orig
    _assert_same(got, ref)
    states = fast.step._states
    assert len(states) == 3 and states.misses == 3, (len(states), states.misses)
    assert all(getattr(st, "graph", None) is not None for st in states.values())
    assert calls["n"] == 12, calls  # one device digest per yielded tensor, none repeated


def test_adam_constant_table_grows_bitwise(gpu, tune, monkeypatch):
    """RowLazyAdam.reserve replaces the step-constant table and drop_graphs
    recaptures every batch — at an epoch's start (a sized loader: size_for) and mid-epoch (a loader
    without len()). Losses, tables, Adam moments and step counts are bitwise those of a run whose
    table never grows; the unsized loader's batch caches grow with it (no LRU churn)."""
    from lgcn_amd import harness

    tune(harness_fused=True)
    U, I, init, arrays = _golden()
    batches = [_B(torch.from_numpy(a).to(gpu)) for a in arrays]
    ref, fast0 = _run(gpu, U, I, init, batches, 5)
    assert fast0.opt.max_steps >= 4096  # never grew
    monkeypatch.setattr(harness, "_MIN_STEPS", 2)
    sized, fast1 = _run(gpu, U, I, init, batches, 5)
    _assert_same(sized, ref)
    assert 15 <= fast1.opt.max_steps < 4096, fast1.opt.max_steps
    monkeypatch.setattr(harness, "_MIN_STATES", 2)
    unsized, fast2 = _run(gpu, U, I, init, lambda: iter(batches), 5)
    _assert_same(unsized, ref)
    assert 15 <= fast2.opt.max_steps < 4096, fast2.opt.max_steps
    states = fast2.step._states
    assert states.capacity >= 4 and states.misses == 3, (states.capacity, states.misses)
