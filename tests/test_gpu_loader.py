"""Device-resident ``Dataset.to_torch(device="cuda")``: the shard is ingested into HBM once
(pinned DMA + arrow_ingest HIP kernel) and batches are slices -- they must equal the host
path's batches, for every feature layout the Ray Data contract allows."""
import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ds():
    from raydp_amd.data import from_pandas
    rng = np.random.default_rng(0)
    n = 1000
    df = pd.DataFrame({"a": rng.normal(size=n), "b": rng.integers(0, 9, n), "c": rng.normal(size=n).astype(np.float32),
                       "y": rng.integers(0, 2, n)})
    return from_pandas([df.iloc[:300], df.iloc[300:700], df.iloc[700:]])   # three blocks


@pytest.mark.parametrize("layout", ["flat", "groups", "per_col_dtypes", "dict"])
def test_device_resident_batches_equal_host_batches(layout):
    ds = _ds()
    kw = dict(label_column="y", label_column_dtype=torch.long, batch_size=64)
    if layout == "flat":
        kw.update(feature_columns=["a", "b", "c"], feature_column_dtypes=torch.float)
    elif layout == "groups":
        kw.update(feature_columns=[["a", "c"], ["b"]], feature_column_dtypes=[torch.float, torch.long])
    elif layout == "per_col_dtypes":
        kw.update(feature_columns=["a", "b", "c"], feature_column_dtypes=[torch.float, torch.float, torch.float])
    else:
        kw.update(feature_columns={"x": ["a", "c"], "k": ["b"]}, feature_column_dtypes={"x": torch.float, "k": torch.long})
    host = list(ds.to_torch(**kw))
    it = ds.to_torch(device="cuda", **kw)
    for _ in range(2):                    # two epochs: the second reuses the resident tensors
        dev = list(it)
        assert len(dev) == len(host)
        for (hf, hl), (df_, dl) in zip(host, dev):
            assert dl.is_cuda and torch.equal(dl.cpu(), hl)
            if isinstance(hf, dict):
                for k in hf:
                    assert df_[k].is_cuda and torch.equal(df_[k].cpu(), hf[k]), k
            elif isinstance(hf, list):
                for a, b in zip(hf, df_):
                    assert b.is_cuda and torch.equal(b.cpu(), a)
            else:
                assert df_.is_cuda and torch.equal(df_.cpu(), hf)
