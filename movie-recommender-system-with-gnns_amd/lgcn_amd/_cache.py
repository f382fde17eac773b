"""Per-batch caches keyed by the batch's CONTENT, not the tensor object.

The reference's loader (PyG DataLoader(batch_size=1, shuffle=True), reference
data/dataset_handler.py:285) collates a new Batch, and so a new edge_index tensor, on every
iteration; keyed by id() every epoch would miss and rebuild what a batch needs (plans, device
copies, captured hipGraphs) while the dead entries piled up. Here an entry is found by:

  1. the tensor object itself (id + weakref + in-place version counter): no hashing, no sync;
  2. else its content key: (device, dtype, shape, 128-bit digest of its bytes) — a CPU tensor is
     hashed in place with XXH3 (BLAKE2b where the xxhash module is absent; a C3 batch's 320 KB in
     ~25 us); a device tensor is digested ON the device (lgcn_digest128: two kernels, then 16 bytes
     to pinned host memory), no copy of the batch. prefetch(t) starts that digest without
     waiting, so a harness that reads its loader one batch ahead (lgcn_amd.harness) finds the
     digest finished when it needs it: no host sync per batch.

Entries live in an LRU of bounded size (least recently used evicted first). The id -> key memo
is shared by every cache (a tensor is hashed at most once while it lives unmodified) and drops the
entries of freed tensors as it grows.

What the memo cannot see: it trusts torch's in-place version counter, and some writes do not bump
it — a write into a torch.from_numpy buffer through numpy, through .data, through DLPack or a raw
data_ptr. A tensor object reused after such a write keeps its old content key (and so the previous
batch's plans and captured graph). A loader that refills one buffer that way must hand over a new
tensor object per batch (a view or a clone), or call forget(t) after each refill.
"""
from __future__ import annotations

import collections
import hashlib
import weakref

import torch

try:  # ~35x faster than BLAKE2b on a batch's bytes (measured: 25 vs 860 us for 320 KB)
    import xxhash

    def _digest(buf) -> bytes:
        return xxhash.xxh3_128(buf).digest()
except ImportError:  # pragma: no cover - xxhash ships with the image
    def _digest(buf) -> bytes:
        return hashlib.blake2b(buf, digest_size=16).digest()


class _PendingDigest:
    """A device digest in flight: 16 bytes landing in a pinned host slot behind an event."""

    __slots__ = ("ring", "slot", "value")

    def __init__(self, ring, slot):
        self.ring, self.slot, self.value = ring, slot, None

    def result(self) -> bytes:
        if self.value is None:
            ring, s = self.ring, self.slot
            ring.events[s].synchronize()
            self.value = ring.host[s].numpy().tobytes()
            if ring.owner[s] is self:
                ring.owner[s] = None
        return self.value


class _DigestRing:
    """Per device: the digests' side stream, workspace and a ring of (device out, pinned host slot,
    event) — preallocated, so a digest costs two launches, one copy and one event record on the
    host (no allocation). A slot still owned by an uncollected digest is collected before reuse."""

    SLOTS = 16

    def __init__(self, dev):
        from . import _ffi

        self.stream = torch.cuda.Stream(dev)
        self.ws = torch.empty(2 * _ffi.DIGEST_BLOCKS, dtype=torch.int64, device=dev)
        self.out = torch.empty((self.SLOTS, 2), dtype=torch.int64, device=dev)
        self.host = torch.empty((self.SLOTS, 2), dtype=torch.int64, pin_memory=True)
        self.events = [torch.cuda.Event() for _ in range(self.SLOTS)]
        self.owner = [None] * self.SLOTS
        self.next = 0


_DIGEST_RINGS: dict = {}


def _device_digest_start(t: torch.Tensor) -> _PendingDigest:
    """lgcn_digest128 of a device tensor's bytes, enqueued on a side stream that waits for the
    current stream's work so far (the tensor's producer) — the current stream goes on with the
    caller's work (a training step) while the digest runs beside it; no host wait."""
    from . import _ffi

    lib = _ffi.load()
    dev = t.device
    ring = _DIGEST_RINGS.get(dev)
    if ring is None:
        ring = _DIGEST_RINGS[dev] = _DigestRing(dev)
    s = ring.next
    ring.next = (s + 1) % ring.SLOTS
    if ring.owner[s] is not None:  # an uncollected digest still owns the slot: collect it first
        ring.owner[s].result()
    stream = ring.stream
    stream.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(stream):
        c = t.detach().contiguous()
        if c.data_ptr() % 8:  # a view at an odd byte offset: digest an aligned copy of the same bytes
            c = c.clone()
        nbytes = c.numel() * c.element_size()
        _ffi.check(lib.lgcn_digest128(c.data_ptr() if nbytes else None, nbytes, ring.ws.data_ptr(), ring.ws.numel(),
                                      ring.out[s].data_ptr(), _ffi.stream_of(dev)), "lgcn_digest128")
        ring.host[s].copy_(ring.out[s], non_blocking=True)
        ring.events[s].record(stream)
    # the caching allocator must not hand the tensor's blocks out again before the side stream is done
    c.record_stream(stream)
    p = _PendingDigest(ring, s)
    ring.owner[s] = p
    return p


def _key_parts(t: torch.Tensor) -> tuple:
    return (str(t.device), str(t.dtype), tuple(t.shape))


def content_key(t: torch.Tensor, extra: tuple = ()) -> tuple:
    """(device, dtype, shape, digest of the bytes, *extra): equal for tensors of equal content."""
    if t.device.type != "cpu":
        return (*_key_parts(t), _device_digest_start(t).result(), *extra)
    host = t.detach().contiguous()
    digest = _digest(host.numpy().view("uint8").data if host.numel() else b"")
    return (*_key_parts(t), digest, *extra)


# id(tensor) -> (weakref, version, content key): shared by every cache, so a tensor is hashed once
_KEYS: dict[int, tuple[weakref.ref, int, tuple]] = {}


def _version(t: torch.Tensor):
    """The in-place version counter, or None for an inference tensor (no counter: never memoised)."""
    try:
        return t._version
    except RuntimeError:
        return None


def _remember(t: torch.Tensor, ver, key) -> None:
    _KEYS[id(t)] = (weakref.ref(t), ver, key)
    if len(_KEYS) > 64 and len(_KEYS) % 64 == 0:  # amortised: drop the entries of freed tensors
        for k in [k for k, (r, _, _) in _KEYS.items() if r() is None]:
            del _KEYS[k]


def prefetch(t: torch.Tensor) -> None:
    """Start t's content key without waiting (a device tensor's digest is enqueued on the current
    stream); tensor_key(t) later collects it. A no-op for CPU tensors, inference tensors and
    tensors whose key is memoised already."""
    ver = _version(t)
    if t.device.type == "cpu" or ver is None:
        return
    hit = _KEYS.get(id(t))
    if hit is not None and hit[0]() is t and hit[1] == ver:
        return
    _remember(t, ver, (_key_parts(t), _device_digest_start(t)))


def tensor_key(t: torch.Tensor) -> tuple:
    """content_key(t), memoised on the tensor object while it lives and is not modified in place."""
    ver = _version(t)
    hit = _KEYS.get(id(t))
    if hit is not None and ver is not None:
        ref, v, key = hit
        if ref() is t and v == ver:
            if isinstance(key, tuple) and len(key) == 2 and isinstance(key[1], _PendingDigest):
                key = (*key[0], key[1].result())  # a prefetched digest: collect it
                _KEYS[id(t)] = (ref, v, key)
            return key
    key = content_key(t)
    if ver is not None:
        _remember(t, ver, key)
    return key


def forget(t: torch.Tensor) -> None:
    """Drop t's memoised key (after a write the version counter does not see)."""
    hit = _KEYS.get(id(t))
    if hit is not None and hit[0]() is t:
        del _KEYS[id(t)]


def _memo_hit(t: torch.Tensor) -> bool:
    """t's key is memoised from an earlier lookup of this object (a prefetched, not yet collected
    digest is a content lookup, not an object hit)."""
    hit = _KEYS.get(id(t))
    return (hit is not None and hit[0]() is t and hit[1] == _version(t)
            and not (len(hit[2]) == 2 and isinstance(hit[2][1], _PendingDigest)))


class ContentLRU:
    """value = cache.get(t, build, extra=()): the value built for a tensor of t's content (and the
    same `extra`), building it with build() on a miss."""

    def __init__(self, capacity: int):
        if capacity < 1:
            raise ValueError("capacity must be >= 1")
        self.capacity = int(capacity)
        self._values: "collections.OrderedDict[tuple, object]" = collections.OrderedDict()
        self.hits_object = self.hits_content = self.misses = 0

    @staticmethod
    def key_of(t: torch.Tensor, extra: tuple = ()) -> tuple:
        return tensor_key(t) + tuple(extra)

    def __contains__(self, key: tuple) -> bool:
        return key in self._values

    def get(self, t: torch.Tensor, build, extra: tuple = ()):
        memo = _memo_hit(t)
        key = self.key_of(t, extra)
        if key in self._values:
            self._values.move_to_end(key)
            if memo:
                self.hits_object += 1
            else:
                self.hits_content += 1
            return self._values[key]
        self.misses += 1
        value = build()
        self._values[key] = value
        while len(self._values) > self.capacity:
            self._values.popitem(last=False)
        return value

    def values(self):
        return list(self._values.values())

    def resize(self, capacity: int) -> None:
        self.capacity = max(1, int(capacity))
        while len(self._values) > self.capacity:
            self._values.popitem(last=False)

    def clear(self) -> None:
        self._values.clear()

    def __len__(self) -> int:
        return len(self._values)
