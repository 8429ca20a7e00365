"""Legacy torch data adapters (reference python/raydp/torch/torch_ml_dataset.py) and the
exception hierarchy (RayDPException.scala)."""
import pyarrow as pa
import pytest
import torch

from raydp_amd.data.dataset import Dataset
from raydp_amd.exceptions import AppMasterError, RayDPException
from raydp_amd.torch.torch_ml_dataset import PrefetchedDataLoader, TorchMLDataset


def _ds():
    return Dataset([pa.table({"x": [float(i) for i in range(j * 10, j * 10 + 10)]}) for j in range(3)])


def test_torch_ml_dataset_blocks_and_len():
    ds = TorchMLDataset(_ds(), lambda pdf: torch.tensor(pdf["x"].values), shuffle=True, shuffle_seed=3)
    assert len(ds) == 30
    got = torch.cat(list(ds))
    assert sorted(got.tolist()) == [float(i) for i in range(30)]


def test_prefetched_loader_order_len_and_reuse():
    base = [torch.full((4,), float(i)) for i in range(7)]
    pl = PrefetchedDataLoader(base, max_size=2, device="cpu")
    assert len(pl) == 7
    for _ in range(2):  # re-iterable
        assert [int(b[0]) for b in pl] == list(range(7))
    # stopping early then restarting does not hang
    it = iter(pl)
    next(it)
    assert [int(b[0]) for b in pl] == list(range(7))


def test_prefetched_loader_propagates_errors():
    def gen():
        yield torch.zeros(1)
        raise ValueError("boom")

    class L:
        def __iter__(self):
            return gen()

        def __len__(self):
            return 2
    with pytest.raises(ValueError):
        list(PrefetchedDataLoader(L()))


def test_exception_hierarchy():
    assert issubclass(AppMasterError, RayDPException)
