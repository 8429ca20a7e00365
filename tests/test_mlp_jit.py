"""Per-model specialised fused-MLP kernels (raydp_amd/ops/mlp_jit.py) on the CPU: the generated
translation unit carries every entry point the launcher looks up (single-workgroup step,
multi-workgroup step, evaluation, persistent epoch), compiles for gfx950 without spilling, and
the cache key follows the kernel headers."""
import os
import subprocess

import pytest
import torch
import torch.nn as nn

from raydp_amd.ops import mlp_jit


def _nyc():
    import __graft_entry__ as g
    return g._nyc_model()


def _trainer(model, batch, loss=None):
    from raydp_amd.models.mlp_spec import extract_mlp_spec
    from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
    return FusedMLPTrainer(extract_mlp_spec(model), optimizer_config(torch.optim.Adam(model.parameters(), lr=1e-3)),
                           loss_code(loss or nn.SmoothL1Loss()), batch, None, layout_only=True)


def test_source_has_every_entry_point_the_launcher_loads():
    src = mlp_jit.generate_source(_trainer(_nyc(), 4096).desc, 4)
    for k in ("rx_jit_step(", "rx_jit_step_mw(", "rx_jit_eval(", "rx_jit_persist("):
        assert f"void {k}" in src, k
    assert "mlp_train_step_mw_body<JitCfg, RX_MT>" in src


def test_batch_wider_than_a_workgroup_takes_several_workgroups():
    tr = _trainer(_nyc(), 4096)
    assert tr.G > 1 and tr.G * 16 * tr.mt >= 4096
    assert _trainer(_nyc(), 64).G == 1


def test_cache_key_changes_with_the_source():
    a = mlp_jit._key(mlp_jit.generate_source(_trainer(_nyc(), 64).desc, 4))
    b = mlp_jit._key(mlp_jit.generate_source(_trainer(_nyc(), 4096).desc, 4))
    assert a != b and len(a) == 24


@pytest.mark.skipif(not os.path.exists(mlp_jit._hipcc()), reason="hipcc not installed")
def test_specialised_kernels_compile_for_gfx950_without_scratch(tmp_path):
    src = mlp_jit.generate_source(_trainer(_nyc(), 4096).desc, 4)
    cpp = tmp_path / "k.hip"
    cpp.write_text(src)
    r = subprocess.run([mlp_jit._hipcc(), "--genco", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-munsafe-fp-atomics", "-I", mlp_jit.CSRC_HIP, str(cpp), "-o", str(tmp_path / "k.hsaco"),
                        "-Rpass-analysis=kernel-resource-usage"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    names, scratch = [], {}
    for line in r.stdout.splitlines():
        if "Function Name:" in line:
            names.append(line.split("Function Name:")[1].split("[")[0].strip())
        elif "ScratchSize" in line and names:
            scratch[names[-1]] = int(line.split(":")[-1].split("[")[0].strip())
    # the specialised step kernels keep every value in registers (the generic, run-time
    # descriptor kernels spill: 348 / 736 B per lane for the single- / multi-workgroup step)
    assert scratch.get("rx_jit_step") == 0 and scratch.get("rx_jit_step_mw") == 0, scratch
