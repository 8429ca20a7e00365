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


def test_fused_optimizer_policy_patches_and_restores_torch_steps():
    """gpu_policy.fused_optimizers: inside, torch's Adam / SGD classes step through the policy
    (CPU parameters: declined once, then torch's own step, with its step hooks); an optimizer
    built inside does not re-wrap the class step; on exit the classes have torch's hooked step."""
    import torch
    from raydp_amd.train.gpu_policy import fused_optimizers
    m = torch.nn.Linear(3, 2)
    ref = torch.nn.Linear(3, 2)
    ref.load_state_dict(m.state_dict())
    x = torch.randn(5, 3)
    o_ref = torch.optim.Adam(ref.parameters(), lr=0.1)
    ref(x).sum().backward()
    o_ref.step()
    with fused_optimizers(True):
        inside = torch.optim.Adam.__dict__["step"]
        o = torch.optim.Adam(m.parameters(), lr=0.1)
        hooked = []
        o.register_step_post_hook(lambda *a: hooked.append(1))
        m(x).sum().backward()
        o.step()
        assert torch.optim.Adam.__dict__["step"] is inside      # not re-wrapped by the new optimizer
        assert o.__dict__.get("_raydp_torch_step") and hooked == [1]
    assert torch.optim.Adam.__dict__["step"] is not inside and getattr(torch.optim.Adam.step, "hooked", False)
    for a, b in zip(ref.parameters(), m.parameters()):
        assert torch.equal(a, b)
    with fused_optimizers(False):
        assert torch.optim.Adam.__dict__["step"] is not inside
