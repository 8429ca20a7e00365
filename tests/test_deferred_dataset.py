"""``Dataset.deferred`` (raydp_amd/data/dataset.py): a dataset whose blocks are still being
produced. Operations that only need the blocks later stay lazy (``random_shuffle`` -- what the
estimator applies before splitting shards for spawned workers), a failure surfaces as the
original error on every access, and the lazy result equals the eager one."""
import concurrent.futures as cf
import threading

import pyarrow as pa
import pytest

from raydp_amd.data.dataset import Dataset, DeferredDatasetError


def _ds(n=100, blocks=4):
    t = pa.table({"x": list(range(n)), "y": [float(i) * 0.5 for i in range(n)]})
    per = n // blocks
    return Dataset([t.slice(i * per, per) for i in range(blocks)], t.schema)


def test_random_shuffle_of_a_deferred_dataset_is_lazy_and_equal_to_eager():
    fut = cf.Future()
    lazy = Dataset.deferred(fut).random_shuffle(seed=7)
    assert lazy._pending is not None          # nothing resolved yet
    fut.set_result(_ds())
    eager = _ds().random_shuffle(seed=7)
    assert lazy.to_arrow().equals(eager.to_arrow())
    assert lazy.num_blocks() == eager.num_blocks()


def test_lazy_shuffle_resolves_once_across_threads():
    fut = cf.Future()
    calls = []
    src = _ds()

    class Counting:
        def result(self):
            calls.append(1)
            return fut.result()
    lazy = Dataset.deferred(Counting()).random_shuffle(seed=1)
    out = []
    ts = [threading.Thread(target=lambda: out.append(lazy.count())) for _ in range(4)]
    for t in ts:
        t.start()
    fut.set_result(src)
    for t in ts:
        t.join()
    assert out == [100] * 4 and len(calls) == 1


def test_failed_source_raises_its_own_error_through_the_lazy_shuffle():
    fut = cf.Future()
    fut.set_exception(KeyError("source failed"))
    lazy = Dataset.deferred(fut).random_shuffle(seed=3)
    for _ in range(2):
        with pytest.raises(DeferredDatasetError) as ei:
            lazy.count()
        # the parent's failure, not a DeferredDatasetError wrapped in another
        assert isinstance(ei.value.original, KeyError)


def test_equal_split_references_blocks_instead_of_copying(runtime_local):
    """Equal shards are slices of the object-store blocks (a few ids when pickled to a worker),
    with the same rows, in the same order, as slicing the concatenated dataset."""
    import pickle
    import pyarrow as pa
    from raydp_amd import runtime
    from raydp_amd.data.dataset import BlockSlice, Dataset
    blocks = [pa.table({"x": list(range(s, s + k))}) for s, k in ((0, 7), (7, 13), (20, 5), (25, 11))]
    ds = Dataset([runtime.put(t) for t in blocks])
    whole = pa.concat_tables(blocks)
    for n in (1, 2, 3, 4, 5):
        shards = ds.split(n, equal=True)
        per = whole.num_rows // n
        for i, sh in enumerate(shards):
            assert all(isinstance(b, BlockSlice) for b in sh._blocks)
            assert len(pickle.dumps(sh)) < 2048
            back = pickle.loads(pickle.dumps(sh))
            assert back.to_arrow().column("x").to_pylist() == whole.slice(i * per, per).column("x").to_pylist()


def test_shuffle_of_store_blocks_is_a_gather_with_the_materialised_rows(runtime_local):
    """random_shuffle over object-store blocks gives gathers (row numbers over the blocks, no row
    copies on the driver) holding the same rows, order and block sizes as the materialised
    shuffle; equal shards of it pickle to ids + row numbers and resolve to the same rows."""
    import pickle
    import numpy as np
    import pyarrow as pa
    from raydp_amd import runtime
    from raydp_amd.data.dataset import BlockGather, Dataset, _split
    blocks = [pa.table({"x": list(range(s, s + k)), "y": [float(v) * 0.5 for v in range(s, s + k)]})
              for s, k in ((0, 7), (7, 13), (20, 5), (25, 11))]
    ds = Dataset([runtime.put(t) for t in blocks])
    whole = pa.concat_tables(blocks)
    sh = ds.random_shuffle(seed=11)
    assert all(isinstance(b, BlockGather) for b in sh._blocks) and sh.num_blocks() == 4
    perm = np.random.default_rng(11).permutation(whole.num_rows)
    want = whole.take(pa.array(perm))
    assert sh.count() == whole.num_rows
    assert sh.to_arrow().to_pylist() == want.to_pylist()
    assert [len(b) for b in sh._blocks] == [t.num_rows for t in _split(want, 4)]
    for n in (2, 3):
        per = whole.num_rows // n
        for i, part in enumerate(sh.split(n, equal=True)):
            blob = pickle.dumps(part)
            assert len(blob) < 2048
            assert pickle.loads(blob).to_arrow().to_pylist() == want.slice(i * per, per).to_pylist()
    # inline (not store-resident) blocks keep the materialised shuffle
    inline = Dataset(blocks).random_shuffle(seed=11)
    assert inline.to_arrow().to_pylist() == want.to_pylist()


def test_gather_shuffle_edge_shapes(runtime_local):
    """More blocks than rows, and more shards than rows: empty gathers resolve to empty tables of
    the schema; the rows are all still there exactly once."""
    import pickle
    import pyarrow as pa
    from raydp_amd import runtime
    from raydp_amd.data.dataset import Dataset
    blocks = [pa.table({"x": [1, 2]}), pa.table({"x": [3]})]
    ds = Dataset([runtime.put(t) for t in blocks]).random_shuffle(seed=3, num_blocks=5)
    assert ds.num_blocks() == 5 and ds.count() == 3
    assert sorted(ds.to_arrow().column("x").to_pylist()) == [1, 2, 3]
    shards = ds.split(4, equal=True)
    assert all(pickle.loads(pickle.dumps(s)).count() == 0 for s in shards)   # 3 rows // 4 = 0 each
    shards = ds.split(3, equal=True)
    got = sorted(v for s in shards for v in pickle.loads(pickle.dumps(s)).to_arrow().column("x").to_pylist())
    assert got == [1, 2, 3]
