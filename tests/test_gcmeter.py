"""raydp_amd.utils.gcmeter: collector time inside a region, and the long-lived-state freeze."""
import gc

from raydp_amd.utils.gcmeter import GcMeter, freeze_long_lived


def test_gc_meter_counts_collections_in_region_only():
    gc.collect()
    with GcMeter() as m:
        gc.collect(0)
        gc.collect(2)
    s = m.summary()
    assert s["collections_by_generation"][0] >= 1 and s["collections_by_generation"][2] >= 1
    assert s["gc_ms"] >= s["gc_max_ms"] >= 0.0
    before = list(m.collections)
    gc.collect()                      # outside the region: not counted
    assert m.collections == before
    assert m._cb not in gc.callbacks


def test_freeze_moves_live_objects_out_of_collections():
    keep = [[i] for i in range(1000)]
    try:
        n = freeze_long_lived()
        assert n >= len(keep)
        assert gc.get_freeze_count() == n
    finally:
        gc.unfreeze()
    assert gc.get_freeze_count() == 0


def test_init_spark_freezes_driver_heap(monkeypatch):
    """spark.ray.mi355x.driver_gc_freeze: the objects alive once the session is up are out of
    the collector's reach (a full collection afterwards walks only what the job creates)."""
    import raydp_amd
    gc.unfreeze()
    spark = raydp_amd.init_spark("gc-freeze", 1, 1, "500M")
    try:
        assert gc.get_freeze_count() > 10000
        assert spark.range(0, 10).count() == 10
    finally:
        raydp_amd.stop_spark()
    # stop_spark hands the frozen objects back to the collector
    assert gc.get_freeze_count() == 0
