"""Host-side planning of the persistent DLRM step (raydp_amd/ops/dlrm_step.py) -- no GPU needed:
the descriptor ABI against the compiled library, the tile planner, the configuration gate and
the LDS budget of every phase for the reference notebook's model (examples/pytorch_dlrm.ipynb
cells 9 and 14) at every supported batch."""
import ctypes

import pytest
import torch

from raydp_amd.models.dlrm import Dlrm
from raydp_amd.ops import dlrm_step as ds


def _model(tables=26, rows=100, top=(1024, 1024, 512, 256, 1)):
    torch.manual_seed(0)
    return Dlrm(13, [rows] * tables, [512, 128, 32], list(top), 32)


def test_descriptor_abi_matches_the_library():
    L = ds._lib()
    assert L.rx_dlrm_desc_size() == ctypes.sizeof(ds.DlrmDesc)
    assert L.rx_dlrm_gspec_size() == ctypes.sizeof(ds.GSpec)
    assert L.rx_dlrm_phase_size() == ctypes.sizeof(ds.Phase)
    assert L.rx_dlrm_max_phases() == ds.MAXPH


@pytest.mark.parametrize("G", [32, 64, 128, 256])
def test_plan_tiles_divide_every_gemm_of_the_notebook_model(G):
    # the notebook's top tower at batch 128: forward, paired dgrad + wgrad of each layer
    B = 128
    shapes = [[(B, 1024, 384)], [(B, 1024, 1024)], [(B, 512, 1024)], [(B, 256, 512)],
              [(B, 512, 256), (256, 512, B)], [(B, 1024, 512), (512, 1024, B)],
              [(B, 1024, 1024), (1024, 1024, B)], [(B, 384, 1024), (1024, 384, B)]]
    for ph in shapes:
        tiles = ds.plan_tiles(ph, G)
        assert len(tiles) == len(ph)
        for (M, N, _), (tm, tn) in zip(ph, tiles):
            assert (tm, tn) in ds._TILES and M % tm == 0 and N % tn == 0


def test_plan_tiles_rejects_an_undividable_shape():
    with pytest.raises(ValueError):
        ds.plan_tiles([(100, 64, 32)], 64)


def test_plan_prefers_one_round_over_fat_tiles_when_the_grid_is_wide():
    # 128 x 1024 forward on 128 workgroups: 128 jobs of 32 x 32 beat 32 jobs of 64 x 64
    (tm, tn), = ds.plan_tiles([(128, 1024, 1024)], 128)
    assert (128 // tm) * (1024 // tn) <= 128
    (tm2, tn2), = ds.plan_tiles([(128, 1024, 1024)], 16)
    assert tm2 * tn2 >= tm * tn      # a narrow grid takes fatter tiles


def test_supported_gates_the_notebook_configuration():
    m = _model()
    sgd = torch.optim.SGD(m.parameters(), lr=0.1)
    bce = torch.nn.BCEWithLogitsLoss()
    assert ds.supported(m, sgd, bce, 128) is None
    assert "batch" in ds.supported(m, sgd, bce, 100)
    assert "batch" in ds.supported(m, sgd, bce, 512)
    assert "optimizer" in ds.supported(m, torch.optim.Adam(m.parameters()), bce, 128)
    assert "momentum" in ds.supported(m, torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9), bce, 128)
    assert "loss" in ds.supported(m, sgd, torch.nn.MSELoss(), 128)
    assert "not a Dlrm" in ds.supported(torch.nn.Linear(2, 2), sgd, bce, 128)
    # the last layer's input must fit the one-pass head (<= 512 features)
    wide = _model(top=(1024, 1024, 1024, 1))
    assert ds.supported(wide, torch.optim.SGD(wide.parameters(), lr=0.1), bce, 128) is not None
    # two learning rates
    m2 = _model()
    groups = [{"params": list(m2.bottom_mlp.parameters()), "lr": 0.1},
              {"params": [p for n, p in m2.named_parameters() if not n.startswith("bottom_mlp")], "lr": 0.2}]
    assert "learning rates" in ds.supported(m2, torch.optim.SGD(groups, lr=0.1), bce, 128)


@pytest.mark.parametrize("B", [32, 64, 128, 256])
def test_every_phase_fits_the_lds_of_one_workgroup(B):
    """The descriptor and LDS plan of a CPU-resident model (no launch): the largest phase fits
    gfx950's 160 KB of LDS per workgroup."""
    m = _model()
    st = ds.DlrmStep.__new__(ds.DlrmStep)
    st.model, st.lr, st.B, st.dev, st.G = m, 0.1, B, torch.device("cpu"), 128
    st.bot = m.bottom_mlp.linears
    st.top = m.top_mlp.linears + [m.out]
    st.F = len(m.embeddings.table_sizes) + 1
    st.D = m.embedding_dim
    st.ZP = ds._ru(st.D + st.F * (st.F - 1) // 2 + 1, 32)
    keep = st._keep = []

    def buf(*shape, dtype=torch.bfloat16):
        t = torch.zeros(*shape, dtype=dtype)
        keep.append(t)
        return t
    st.layers = [(lin, ds._ru(lin.in_features, 32), buf(2, lin.out_features, ds._ru(lin.in_features, 32)),
                  buf(2, ds._ru(lin.in_features, 32), lin.out_features)) for lin in st.bot + st.top[:-1]]
    nb = len(st.bot)
    st.XdT = buf(st.layers[0][1], B)
    st.H = [(buf(B, l.out_features), buf(l.out_features, B)) if i < nb - 1 else (None, None)
            for i, l in enumerate(st.bot)]
    st.ximg = buf(B, 32, st.D)
    st.Z, st.ZT = buf(B, st.ZP), buf(st.ZP, B)
    topm = st.top[:-1]
    st.A = [(buf(B, l.out_features), buf(l.out_features, B) if i < len(topm) - 1 else None)
            for i, l in enumerate(topm)]
    st.dA = [(buf(B, l.out_features), buf(l.out_features, B)) for l in topm]
    st.dZ = buf(B, st.ZP, dtype=torch.float32)
    st.dmlp, st.dmlpT = buf(B, st.D), buf(st.D, B)
    st.dH = [(buf(B, l.in_features), buf(l.in_features, B)) for l in st.bot[1:]]
    st.logits = buf(B, dtype=torch.float32)
    st.loss_acc = buf(1, dtype=torch.float64)
    st.step_loss = buf(1, dtype=torch.float32)
    st.head_ld = ds._ru(st.top[-1].in_features + 4, 4)
    st.head_part = buf(B // 16, st.head_ld, dtype=torch.float32)
    st.ctl = buf(8, dtype=torch.int32)
    st.ticks = 1
    st.desc = ds.DlrmDesc()
    st._build_phases()
    kinds = [st.desc.ph[k].kind for k in range(st.desc.nph)]
    assert kinds[0] == ds.PH_BOTTOM and ds.PH_HEAD in kinds and ds.PH_IBWD in kinds
    assert st.desc.nph <= ds.MAXPH
    assert st._lds_bytes() <= 160 * 1024
