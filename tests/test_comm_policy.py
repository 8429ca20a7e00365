"""DDP comm-stream policy (raydp_amd/ops/comm.py comm_stream_wanted): ``auto`` overlaps the
bucket reductions with backward only when no two ranks share a GPU -- ranks time-sharing one
device measured 5-8x slower with the comm stream (profiles/r4_ddp_bucket_sweep.txt). gloo, CPU."""
import os

from test_multirank import _init, _spawn


def _policy_main(rank, world, port, q, shared, setting):
    import raydp_amd.ops.comm as C
    _init(rank, world, port)
    try:
        # rank r's "GPU": all ranks on one device, or one device each
        C._device_key = lambda: ("host", 0 if shared else rank)
        if setting is None:
            os.environ.pop("RAYDP_DDP_COMM_STREAM", None)
        else:
            os.environ["RAYDP_DDP_COMM_STREAM"] = setting
        q.put((rank, C.comm_stream_wanted()))
    finally:
        import torch.distributed as dist
        dist.destroy_process_group()


def test_auto_overlaps_only_when_every_rank_has_its_own_gpu():
    assert [r[1] for r in _spawn(_policy_main, 2, False, None)] == [True, True]
    assert [r[1] for r in _spawn(_policy_main, 3, True, None)] == [False, False, False]


def test_explicit_settings_win_over_the_device_layout():
    assert [r[1] for r in _spawn(_policy_main, 2, True, "on")] == [True, True]
    assert [r[1] for r in _spawn(_policy_main, 2, False, "0")] == [False, False]


def test_without_a_process_group_auto_means_on(monkeypatch):
    import raydp_amd.ops.comm as C
    monkeypatch.delenv("RAYDP_DDP_COMM_STREAM", raising=False)
    assert C.comm_stream_wanted() is True
    monkeypatch.setenv("RAYDP_DDP_COMM_STREAM", "off")
    assert C.comm_stream_wanted() is False
