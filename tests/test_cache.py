"""lgcn_amd._cache: per-batch caches found by the tensor object or by its content (ADVICE r4:
the reference's PyG DataLoader collates a new edge_index tensor every epoch, reference
data/dataset_handler.py:285). CPU only."""
import torch

from lgcn_amd._cache import ContentLRU, content_key, tensor_key


def test_content_key_equal_for_equal_content_and_differs_otherwise():
    a = torch.arange(20).view(2, 10)
    assert content_key(a) == content_key(a.clone())
    assert content_key(a) != content_key(a + 1)
    assert content_key(a) != content_key(a.view(4, 5))  # shape is part of the key
    assert content_key(a) != content_key(a.to(torch.int32))  # dtype too
    assert content_key(a.t()) == content_key(a.t().contiguous())  # layout is not
    assert content_key(torch.empty(2, 0, dtype=torch.int64)) == content_key(torch.empty(2, 0, dtype=torch.int64))


def test_lru_hits_by_object_then_by_content_and_evicts_least_recent():
    c = ContentLRU(2)
    a = torch.arange(10).view(2, 5)
    builds = []

    def build(tag):
        def f():
            builds.append(tag)
            return tag
        return f

    assert c.get(a, build("A")) == "A"
    assert c.get(a, build("A2")) == "A" and c.hits_object == 1  # the same object: no hashing
    assert c.get(a.clone(), build("A3")) == "A" and c.hits_content == 1  # a new tensor, same edges
    b = torch.arange(10, 20).view(2, 5)
    assert c.get(b, build("B")) == "B"
    c.get(a, build("A4"))  # refresh A: B is now the least recently used
    d = torch.arange(20, 30).view(2, 5)
    c.get(d, build("D"))
    assert len(c) == 2 and c.get(b.clone(), build("B2")) == "B2"  # B was evicted, rebuilt
    assert builds == ["A", "B", "D", "B2"]


def test_in_place_change_is_a_new_key():
    c = ContentLRU(4)
    a = torch.arange(6).view(2, 3)
    assert c.get(a, lambda: 1) == 1
    a.add_(1)  # version counter moves: the memoised key is not trusted
    assert c.get(a, lambda: 2) == 2
    assert tensor_key(a) == content_key(a)


def test_extra_key_parts_separate_entries():
    c = ContentLRU(4)
    a = torch.arange(6).view(2, 3)
    assert c.get(a, lambda: "n5", extra=(5, 0)) == "n5"
    assert c.get(a, lambda: "n7", extra=(7, 0)) == "n7"
    assert c.get(a.clone(), lambda: "x", extra=(5, 0)) == "n5"


def test_inference_tensors_are_keyed_by_content():
    c = ContentLRU(4)
    with torch.inference_mode():
        a = torch.arange(6).view(2, 3)
    assert c.get(a, lambda: 1) == 1
    assert c.get(a.clone(), lambda: 2) == 1
