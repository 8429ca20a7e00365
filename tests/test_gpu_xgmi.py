"""One-shot xGMI all-reduce (csrc/comm/xgmi_allreduce.hip) with two ranks sharing ONE GPU.

gpurun gives one MI355X, so the peer mapping is exercised between two processes on the same
device (hipIpcOpenMemHandle of a region owned by another process); the flag protocol, the
double-buffered slots, the rank-order summation and the fused reduce+Adam kernel are the same
code that runs across 8 GPUs. Bootstrap (IPC handle exchange) goes over gloo.
"""
import multiprocessing as mp
import os
import sys

import pytest

from raydp_amd.train.trainer import _free_port

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _init(rank, world, port):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)


def _allreduce_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    _init(rank, world, port)
    try:
        from raydp_amd.ops.comm import XgmiComm
        # NYC gradient (194 KB), a 1 MiB bucket, the DLRM dense gradient (8.7 MB), an odd size
        sizes = [48_513, 262_144, 2_177_185, 50_001]
        comm = XgmiComm.create(max(sizes), timeout_s=20.0)
        if comm is None:
            q.put((rank, "create failed", 0.0))
            return
        worst = 0.0
        for it in range(8):
            n = sizes[it % len(sizes)]
            data = [torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + r)).cuda()
                    for r in range(world)]
            want = torch.zeros(n, device="cuda")
            for r in range(world):       # rank order: the kernel's summation order
                want = want + data[r]
            scale = 1.0 / world if it % 2 else 1.0
            if it == 5:
                # unaligned (scalar) path: a view starting one float into its storage
                buf = torch.zeros(n + 1, device="cuda")
                buf[1:] = data[rank]
                t = buf[1:]
            else:
                t = data[rank].clone()
            comm.allreduce_(t, scale)
            torch.cuda.synchronize()
            worst = max(worst, float((t - want * scale).abs().max()))
        q.put((rank, "ok" if comm.error() == 0 else "error word set", worst))
        torch.cuda.synchronize()
        dist.barrier()
        comm.close()
    finally:
        dist.destroy_process_group()


def _nyc(cols=20):
    import torch.nn as nn
    import torch.nn.functional as F

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc1, self.fc2, self.fc3 = nn.Linear(cols, 64), nn.Linear(64, 32), nn.Linear(32, 1)
            self.bn1 = nn.BatchNorm1d(64)

        def forward(self, x):
            return self.fc3(F.relu(self.fc2(self.bn1(F.relu(self.fc1(x))))))

    return M()


def _fused_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import torch.nn as nn
    _init(rank, world, port)
    try:
        from raydp_amd.models.mlp_spec import extract_mlp_spec
        from raydp_amd.ops.comm import XgmiComm
        from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
        dev = torch.device("cuda", 0)
        outs = []
        for mode in ("xgmi", "gloo"):
            torch.manual_seed(0)
            model = _nyc()
            # SGD + momentum: the two paths differ only in the fp32 summation order of dW, which
            # SGD carries through linearly (Adam's first steps are ~lr * sign(g): a near-zero
            # gradient whose sign flips under reordering moves a weight by 2 lr)
            opt = torch.optim.SGD(model.parameters(), lr=1e-2, momentum=0.9)
            tr = FusedMLPTrainer(extract_mlp_spec(model), optimizer_config(opt), loss_code(nn.MSELoss()), 64, dev)
            g = torch.Generator().manual_seed(7 + rank)
            n = 64 * 16
            feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16)
            feats[:, :20] = torch.randn(n, 20, generator=g).to(torch.bfloat16)
            labels = torch.randn(n, 1, generator=g)
            feats, labels = feats.to(dev), labels.to(dev)
            if mode == "xgmi":
                xg = XgmiComm.create(tr.grads.numel(), timeout_s=20.0, host_seq=True)
                if xg is None:
                    q.put((rank, "create failed", None, None))
                    return
                for _ in range(2):
                    tr.train_epoch(feats, labels, n, None, world_size=world, xg=xg)
            else:
                def ar(gr):
                    dist.all_reduce(gr)
                for _ in range(2):
                    tr.train_epoch(feats, labels, n, None, allreduce=ar, world_size=world)
            torch.cuda.synchronize()
            outs.append(tr.params.detach().cpu().clone())
        # replicas must be bit-identical across ranks on the xGMI path
        gathered = [None] * world
        dist.all_gather_object(gathered, outs[0])
        same = all(bool(torch.equal(gathered[0], x)) for x in gathered)
        diff = float((outs[0] - outs[1]).abs().max())
        scale = float(outs[1].abs().max())
        q.put((rank, "ok", same, diff / scale))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(target, world=2, timeout=100):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = sorted(q.get(timeout=timeout) for _ in ps)
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return res


@pytest.mark.parametrize("world", [2, 4, 8])
def test_xgmi_allreduce_ranks_share_one_gpu(world):
    """World 8 is a full MI355X node's fan-out: 7 peer reads per element and 7 remote flag
    writers per region, one launch-wide rendezvous per call, 16-B peer loads (and the scalar
    path for an unaligned buffer), buckets from 194 KB to 8.7 MB, sum and average."""
    res = _run(_allreduce_main, world)
    assert len(res) == world
    for rank, status, worst in res:
        assert status == "ok", (rank, status)
        assert worst < 1e-5, (rank, worst)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_fused_step_loop_with_xgmi_reduce_matches_gloo_allreduce(world):
    res = _run(_fused_main, world)
    for rank, status, same, rel in res:
        assert status == "ok", (rank, status)
        assert same, "replicas diverged across ranks"
        # the xGMI path sums the ranks inside the dW MFMA (rank-concatenated batch), the gloo
        # path adds materialised per-rank dW: fp32 summation order only
        assert rel < 1e-4, (rank, rel)


def _nyc_full(cols=20):
    """The flagship NYC_Model (examples/pytorch_nyctaxi.py): 5 Linear + 4 BatchNorm1d."""
    import torch.nn as nn
    import torch.nn.functional as F

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc1, self.fc2, self.fc3 = nn.Linear(cols, 256), nn.Linear(256, 128), nn.Linear(128, 64)
            self.fc4, self.fc5 = nn.Linear(64, 16), nn.Linear(16, 1)
            self.bn1, self.bn2 = nn.BatchNorm1d(256), nn.BatchNorm1d(128)
            self.bn3, self.bn4 = nn.BatchNorm1d(64), nn.BatchNorm1d(16)

        def forward(self, x):
            x = self.bn1(F.relu(self.fc1(x)))
            x = self.bn2(F.relu(self.fc2(x)))
            x = self.bn3(F.relu(self.fc3(x)))
            x = self.bn4(F.relu(self.fc4(x)))
            return self.fc5(x)
    return M()


def _tiles_main(rank, world, port, q, batch=64, steps=12):
    """The data-parallel fused engine with the gradient exchanged INSIDE the training launches
    (persistent epoch at batch <= 128, the multi-workgroup step's optimizer tasks above), against
    the same trainer with a gloo all-reduce of materialised gradients between launches."""
    import torch
    import torch.distributed as dist
    import torch.nn as nn
    _init(rank, world, port)
    try:
        from raydp_amd.models.mlp_spec import extract_mlp_spec
        from raydp_amd.ops.comm import XgmiComm
        from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
        dev = torch.device("cuda", 0)
        outs, paths, times = [], [], None
        for mode in ("xgmi", "gloo"):
            torch.manual_seed(0)
            model = _nyc_full()
            opt = torch.optim.SGD(model.parameters(), lr=1e-2, momentum=0.9)
            tr = FusedMLPTrainer(extract_mlp_spec(model), optimizer_config(opt), loss_code(nn.SmoothL1Loss()),
                                 batch, dev, world=world)
            tr.record_steps = True
            g = torch.Generator().manual_seed(7 + rank)
            n = batch * steps
            feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16)
            feats[:, :20] = torch.randn(n, 20, generator=g).to(torch.bfloat16)
            labels = torch.randn(n, 1, generator=g) * 3
            feats, labels = feats.to(dev), labels.to(dev)
            perm = torch.randperm(n, generator=torch.Generator().manual_seed(3)).to(torch.int32).to(dev)
            if mode == "xgmi":
                xg = XgmiComm.create(tr.total if tr.G > 1 else tr.grads.numel(), timeout_s=20.0, host_seq=True)
                if xg is None:
                    q.put((rank, "create failed", None, None, None, None))
                    return
                tr.share = xg.share
                if tr._mw_args is not None:
                    tr._mw_args.share = xg.share
                for _ in range(2):
                    tr.train_epoch(feats, labels, n, perm, world_size=world, xg=xg)
                    paths.append(tr.last_path)
                    st = tr.step_times_us()
                    times = st if st is not None else times
            else:
                def ar(gr):
                    # every rank's gradient, summed in rank order from zero: the exchange's own
                    # summation order, so the two paths must agree bit for bit
                    parts = [torch.empty_like(gr) for _ in range(world)]
                    dist.all_gather(parts, gr)
                    acc = torch.zeros_like(gr)
                    for p_ in parts:
                        acc = acc + p_
                    gr.copy_(acc)
                for _ in range(2):
                    tr.train_epoch(feats, labels, n, perm, allreduce=ar, world_size=world)
            torch.cuda.synchronize()
            outs.append(torch.cat([tr.params.detach().cpu(), tr.rstats.detach().cpu()]).clone())
        gathered = [None] * world
        dist.all_gather_object(gathered, outs[0][:tr.total])
        same = all(bool(torch.equal(gathered[0], x)) for x in gathered)
        rel = float((outs[0] - outs[1]).abs().max()) / float(outs[1].abs().max())
        q.put((rank, "ok", same, rel, tuple(paths), None if times is None else float(sorted(times)[len(times) // 2])))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _tiles_b64(rank, world, port, q):
    _tiles_main(rank, world, port, q, batch=64, steps=16)


def _tiles_b1000(rank, world, port, q):
    _tiles_main(rank, world, port, q, batch=1000, steps=6)


def _tiles_b4096(rank, world, port, q):
    _tiles_main(rank, world, port, q, batch=4096, steps=4)


@pytest.mark.parametrize("world,target,path", [(2, "_tiles_b64", "persistent_xgmi_tiles"),
                                               (4, "_tiles_b64", "persistent_xgmi_tiles"),
                                               (8, "_tiles_b64", "persistent_xgmi_tiles"),
                                               (2, "_tiles_b1000", "mw_xgmi_tiles"),
                                               (4, "_tiles_b1000", "mw_xgmi_tiles"),
                                               (8, "_tiles_b1000", "mw_xgmi_tiles"),
                                               (2, "_tiles_b4096", "mw_xgmi_tiles"),
                                               (4, "_tiles_b4096", "mw_xgmi_tiles")])
def test_in_launch_gradient_exchange_matches_gloo_allreduce(world, target, path):
    """World > 1 on the one-GPU engine's kernels: batch 64 trains in the persistent epoch launch
    and batch 1000 / 4096 in the multi-workgroup step, each exchanging per-tile GRADIENTS over
    xGMI inside the launch (the optimizer workgroups meet their peers per 32x32 tile). Replicas
    stay bit-identical, and the parameters and BatchNorm statistics equal those of the same
    trainer fed a gloo all-gather of materialised gradients summed in rank order between
    launches (the exchange's summation order), and the device step time is recorded at
    world > 1. (World 8 at batch 4096 is 8 x 64 step workgroups: more than one GPU holds at once,
    so that shape waits for 8 real GPUs.)"""
    res = _run(globals()[target], world, timeout=200)
    assert len(res) == world
    for rank, status, same, rel, paths, step_us in res:
        assert status == "ok", (rank, status)
        assert all(p == path for p in paths), (rank, paths)
        assert same, "replicas diverged across ranks"
        # persistent: bit-level agreement; multi-workgroup: the local dW is summed over split-K
        # partials in-launch vs one K chain in the materialising kernel (fp32 order only)
        assert rel < (1e-6 if path.startswith("persistent") else 1e-4), (rank, rel)
        assert step_us is not None and step_us > 0, (rank, step_us)


def _ddp_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    _init(rank, world, port)
    try:
        from raydp_amd.ops import comm as C
        from raydp_amd.parallel.ddp import DistributedDataParallel
        res = {}
        for mode in ("auto", "rccl"):   # rccl: BucketAllreduce falls back to dist.all_reduce (gloo here)
            os.environ["RAYDP_ALLREDUCE"] = mode
            torch.manual_seed(0)
            net = torch.nn.Sequential(torch.nn.Linear(20, 64), torch.nn.ReLU(), torch.nn.Linear(64, 1)).cuda()
            ddp = DistributedDataParallel(net)
            used = ddp._allreduce.xg is not None
            opt = torch.optim.SGD(ddp.parameters(), lr=0.05)
            g = torch.Generator().manual_seed(11 + rank)
            for _ in range(5):
                x = torch.randn(32, 20, generator=g).cuda()
                y = torch.randn(32, 1, generator=g).cuda()
                opt.zero_grad()
                torch.nn.functional.mse_loss(ddp(x), y).backward()
                opt.step()
            torch.cuda.synchronize()
            res[mode] = (used, torch.cat([p.detach().reshape(-1) for p in net.parameters()]).cpu())
        os.environ.pop("RAYDP_ALLREDUCE", None)
        gathered = [None] * world
        dist.all_gather_object(gathered, res["auto"][1])
        same = all(bool(torch.equal(gathered[0], t)) for t in gathered)
        diff = float((res["auto"][1] - res["rccl"][1]).abs().max())
        q.put((rank, res["auto"][0], res["rccl"][0], same, diff))
        dist.barrier()
        C.reset_cache()
    finally:
        dist.destroy_process_group()


def test_ddp_small_buckets_take_the_xgmi_path():
    res = _run(_ddp_main)
    for rank, used_xg, used_fallback, same, diff in res:
        assert used_xg and not used_fallback, (rank, used_xg, used_fallback)
        assert same, "DDP replicas diverged"
        assert diff < 1e-5, (rank, diff)


def _fallback_main(rank, world, port, q):
    import types

    import torch
    import torch.distributed as dist
    import torch.nn as nn
    _init(rank, world, port)
    try:
        from raydp_amd.exceptions import CollectiveError
        from raydp_amd.models.mlp_spec import extract_mlp_spec
        from raydp_amd.ops import comm as C
        from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
        from raydp_amd.torch.engine import FusedMLPEngine
        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        model = _nyc()
        opt = torch.optim.Adam(model.parameters(), lr=1e-2)
        tr = FusedMLPTrainer(extract_mlp_spec(model), optimizer_config(opt), loss_code(nn.MSELoss()), 64, dev)
        g = torch.Generator().manual_seed(7 + rank)
        n = 64 * 16
        feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16)
        feats[:, :20] = torch.randn(n, 20, generator=g).to(torch.bfloat16)
        labels = torch.randn(n, 1, generator=g)
        feats, labels = feats.to(dev), labels.to(dev)
        xg = C.XgmiComm.create(tr.grads.numel(), timeout_s=20.0, host_seq=True)
        if xg is None:
            q.put((rank, "create failed", None, None))
            return
        eng = types.SimpleNamespace(trainer=tr, world=world, drop_last=False, xg=xg, ar=None, comm=None,
                                    max_steps=None, shuffle=False, epoch=0, metrics_names=[],
                                    train=types.SimpleNamespace(feats_bf16=feats, labels=labels, n=n))
        eng._res = lambda m: {}
        outcomes = []
        for ep in range(2):
            if ep == 1 and rank == 1:
                xg._inject_error()          # rank 1 "missed a peer" during epoch 1
            try:
                FusedMLPEngine.train_epoch(eng)
                outcomes.append("ok")
            except CollectiveError:
                outcomes.append("collective_error")
        torch.cuda.synchronize()
        # the process dropped the xGMI path: a new communicator is refused on every rank
        again = C.XgmiComm.create(tr.grads.numel(), timeout_s=20.0, host_seq=True)
        q.put((rank, tuple(outcomes), eng.xg is None, again is None))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_xgmi_timeout_on_one_rank_fails_every_rank_in_the_same_epoch():
    """A peer miss on ONE rank reaches every rank through the epoch-end vote (read with the
    metrics, no extra host sync): all ranks raise CollectiveError in the same epoch -- a worker
    failure, so the trainer restarts the group from its newest checkpoint -- and the process
    stops using xGMI."""
    res = _run(_fallback_main)
    for rank, outcomes, dropped, refused in res:
        assert outcomes == ("ok", "collective_error"), (rank, outcomes)
        assert dropped and refused, (rank, dropped, refused)


def _ddp_graph_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import torch.nn as nn
    _init(rank, world, port)
    try:
        from raydp_amd.ops import comm as C
        from raydp_amd.parallel.ddp import DistributedDataParallel
        dev = torch.device("cuda", 0)
        g = torch.Generator().manual_seed(11 + rank)
        xs = [torch.randn(64, 20, generator=g).to(dev) for _ in range(6)]
        ys = [torch.randn(64, 1, generator=g).to(dev) for _ in range(6)]
        outs = {}
        for mode in ("eager", "graph"):
            torch.manual_seed(0)
            net = nn.Sequential(nn.Linear(20, 64), nn.ReLU(), nn.BatchNorm1d(64), nn.Linear(64, 1)).to(dev)
            ddp = DistributedDataParallel(net)
            assert ddp.capturable(), "NYC-sized DDP buckets must ride the capturable one-shot kernel"
            opt = torch.optim.Adam(ddp.parameters(), lr=1e-2, capturable=True)
            sx, sy = torch.zeros_like(xs[0]), torch.zeros_like(ys[0])

            def step():
                ddp.zero_grad()
                loss = nn.functional.mse_loss(ddp(sx), sy)
                loss.backward()
                opt.step()
            # two eager steps on a side stream (optimizer state, workspaces), then capture
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for i in range(2):
                    sx.copy_(xs[i])
                    sy.copy_(ys[i])
                    step()
            torch.cuda.current_stream().wait_stream(side)
            if mode == "eager":
                for i in range(2, 6):
                    sx.copy_(xs[i])
                    sy.copy_(ys[i])
                    step()
            else:
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    step()
                for i in range(2, 6):
                    sx.copy_(xs[i])
                    sy.copy_(ys[i])
                    graph.replay()
            torch.cuda.synchronize()
            outs[mode] = torch.cat([t.detach().reshape(-1) for t in list(net.parameters()) + list(net.buffers())
                                    if t.dtype.is_floating_point]).cpu()
            outs[mode + "_params"] = torch.cat([t.detach().reshape(-1) for t in net.parameters()]).cpu()
        # parameters agree across ranks; BN running stats are rank 0's at every forward's
        # broadcast and then each rank's own batch statistics (torch DDP's broadcast_buffers)
        gathered = [None] * world
        dist.all_gather_object(gathered, outs["graph_params"])
        same_ranks = all(bool(torch.equal(gathered[0], t)) for t in gathered)
        q.put((rank, bool(torch.equal(outs["eager"], outs["graph"])), same_ranks))
        dist.barrier()
        C.reset_cache()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ddp_step_graph_replay_over_xgmi_matches_eager_bitwise(world):
    """A whole DDP step (BN buffer broadcast, backward with the bucket all-reduce, average,
    Adam) captured into one HIP graph and replayed at world > 1 trains bit for bit like the
    eager loop, and every replica stays identical."""
    res = _run(_ddp_graph_main, world)
    for rank, same_as_eager, same_ranks in res:
        assert same_as_eager, f"rank {rank}: graph replay diverged from the eager DDP loop"
        assert same_ranks, "replicas diverged"


def _emb_sync_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    _init(rank, world, port)
    try:
        from raydp_amd.ops.comm import XgmiComm
        from raydp_amd.ops.dlrm_ops import FusedEmbeddings
        dev = torch.device("cuda", 0)
        # the all-gather itself: int64 ids and fp32 rows, rank order
        comm = XgmiComm.create(64 * 27 * 32 + 64, timeout_s=20.0)
        src = torch.arange(10, dtype=torch.int64, device=dev) + 100 * rank
        dst = torch.empty(world, 10, dtype=torch.int64, device=dev)
        comm.allgather_(src, dst)
        gathered_ok = bool(torch.equal(dst.cpu(), torch.stack([torch.arange(10) + 100 * r for r in range(world)])))
        # replicated tables, SGD fused into backward, rows gathered over xGMI
        sizes, D, B, lr = [50, 70, 30], 32, 64, 0.1
        torch.manual_seed(0)
        emb = FusedEmbeddings(sizes, D).to(dev)
        w0 = emb.weight.detach().clone()
        emb.fused_sgd_lr, emb.sync = lr, (comm, world)
        g = torch.Generator().manual_seed(3)
        ids = [torch.stack([torch.randint(0, s, (B,), generator=g) for s in sizes], 1) for _ in range(world)]
        heads = [torch.randn(B, D, generator=g) for _ in range(world)]
        X = emb(heads[rank].to(dev), ids[rank].to(dev))
        (X[:, 1:] ** 2).sum().backward()
        torch.cuda.synchronize()
        # reference: the average over ranks of every rank's sparse gradient, one SGD step
        ref = w0.cpu().clone()
        offs = torch.tensor([0, 50, 120])
        for r in range(world):
            rows = (ids[r] + offs.view(1, -1)).reshape(-1)
            grad_rows = 2 * w0.cpu()[rows]
            ref.index_add_(0, rows, grad_rows, alpha=-lr / world)
        err = float((emb.weight.detach().cpu() - ref).abs().max())
        q.put((rank, gathered_ok, err))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_replicated_embedding_rows_gathered_over_xgmi():
    """DLRM tables replicated over ranks with the fused SGD: every rank applies every rank's
    gradient rows (all-gathered on the device over xGMI) -- the same table as the averaged
    sparse all-reduce of DDP, on every rank."""
    res = _run(_emb_sync_main, 2)
    for rank, gathered_ok, err in res:
        assert gathered_ok, rank
        assert err < 1e-5, (rank, err)


def _sharded_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    _init(rank, world, port)
    try:
        from raydp_amd.ops import comm as C
        from raydp_amd.parallel.embedding_mp import ShardedEmbeddings
        dev = torch.device("cuda", 0)
        # the raw kernel: rank r sends (p + 1) * (r + 2) words to rank p, values tagged by (r, p)
        xg = C.XgmiComm.create(C.XG_BUCKET_MAX_BYTES // 4, timeout_s=20.0)
        send_len = [(p + 1) * (rank + 2) for p in range(world)]
        src = torch.cat([torch.full((n,), float(100 * rank + p)) for p, n in enumerate(send_len)]).to(dev)
        recv_len = [(rank + 1) * (p + 2) for p in range(world)]
        from_off = [sum((q_ + 1) * (p + 2) for q_ in range(rank)) for p in range(world)]
        dst_off = [sum(recv_len[:p]) for p in range(world)]
        dst = torch.full((sum(recv_len),), -1.0, device=dev)
        xg.alltoallv_(src, dst, from_off, recv_len, dst_off)
        want = torch.cat([torch.full((n,), float(100 * p + rank)) for p, n in enumerate(recv_len)])
        raw_ok = bool(torch.equal(dst.cpu(), want))
        # sharded DLRM tables: the xGMI exchanges on the GPU vs gloo all_to_all on the CPU
        sizes, D, B, lr = [50, 70, 30, 90, 20], 32, 48, 0.05
        g = torch.Generator().manual_seed(5 + rank)
        idx = torch.stack([torch.randint(0, s, (B,), generator=g) for s in sizes], 1)
        head = torch.randn(B, D, generator=g)
        res = {}
        for where in ("gpu", "cpu"):
            d = dev if where == "gpu" else torch.device("cpu")
            emb = ShardedEmbeddings(sizes, D, seed=1, fused_sgd_lr=lr, static_batch=True).to(d)
            X = emb(head.to(d), idx.to(d))
            (X[:, 1:] ** 2).sum().backward()
            res[where] = (X.detach().cpu(), emb.weight.detach().cpu(), emb._xg is not None)
        fwd_err = float((res["gpu"][0] - res["cpu"][0]).abs().max())
        w_err = float((res["gpu"][1] - res["cpu"][1]).abs().max())
        # a whole lookup + backward + fused SGD step captured into a HIP graph, replayed
        outs = {}
        for mode in ("eager", "graph"):
            emb = ShardedEmbeddings(sizes, D, seed=1, fused_sgd_lr=lr, static_batch=True).to(dev)
            sh, si = head.to(dev).clone(), idx.to(dev).clone()

            def step():
                X = emb(sh, si)
                (X[:, 1:] ** 2).sum().backward()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                step()
            torch.cuda.current_stream().wait_stream(side)
            if mode == "eager":
                for _ in range(3):
                    step()
            else:
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    step()
                for _ in range(3):
                    graph.replay()
            torch.cuda.synchronize()
            outs[mode] = emb.weight.detach().cpu()
        # (the row SGD adds duplicate rows with float atomics: equal up to summation order)
        q.put((rank, raw_ok, res["gpu"][2], fwd_err, w_err, float((outs["eager"] - outs["graph"]).abs().max())))
        dist.barrier()
        C.reset_cache()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_embeddings_exchange_over_xgmi(world):
    """Table-wise sharded DLRM embeddings (K12): the id, row and row-gradient all-to-alls run
    on the one-shot xGMI kernel -- the same forward output and fused-SGD tables as gloo's
    all_to_all on the CPU -- and a whole lookup + backward step captures into a HIP graph that
    replays like the eager loop."""
    res = _run(_sharded_main, world)
    for rank, raw_ok, used_xg, fwd_err, w_err, graph_err in res:
        assert raw_ok, f"rank {rank}: variable-split all-to-all delivered the wrong words"
        assert used_xg, "the GPU lookup should ride the xGMI all-to-all"
        assert fwd_err < 1e-6 and w_err < 1e-6, (rank, fwd_err, w_err)
        assert graph_err < 1e-6, f"rank {rank}: graph replay diverged from eager ({graph_err})"


def _twoshot_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    _init(rank, world, port)
    try:
        from raydp_amd.ops.comm import XgmiComm
        sizes = [48_516, 262_144, 2_177_188, 50_004]      # multiples of 4 (the two-shot contract)
        comm = XgmiComm.create(max(sizes), timeout_s=20.0)
        if comm is None:
            q.put((rank, "create failed", 0.0, False))
            return
        worst, ran2, outs = 0.0, True, []
        for it in range(10):
            n = sizes[it % len(sizes)]
            data = [torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + r)).cuda()
                    for r in range(world)]
            want = torch.zeros(n, device="cuda")
            for r in range(world):
                want = want + data[r]
            scale = 1.0 / world if it % 2 else 1.0
            t = data[rank].clone()
            # interleave the kernels: one-shot calls consume one sequence number, two-shot three,
            # and the slot parity must still alternate call to call
            if it % 3 == 2:
                comm.allreduce_(t, scale)
            else:
                ran2 = comm.allreduce2_(t, scale) and ran2
            torch.cuda.synchronize()
            worst = max(worst, float((t - want * scale).abs().max()))
            outs.append(t.cpu())
        # an unaligned buffer is refused (the caller falls back to the one-shot kernel)
        buf = torch.zeros(1025, device="cuda")
        refused = not comm.allreduce2_(buf[1:])
        gathered = [None] * world
        dist.all_gather_object(gathered, torch.cat(outs))
        same = all(bool(torch.equal(gathered[0], x)) for x in gathered)
        q.put((rank, "ok" if comm.error() == 0 else "error word set", worst, ran2 and refused and same))
        torch.cuda.synchronize()
        dist.barrier()
        comm.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_xgmi_twoshot_allreduce_interleaved_with_oneshot(world):
    """The all-pairs two-shot kernel (reduce-scatter + all-gather over the same slots) gives the
    rank-order sum, bit-identical on every rank, including when its calls alternate with one-shot
    calls on the same communicator (slot parity and sequence numbers stay consistent)."""
    res = _run(_twoshot_main, world)
    assert len(res) == world
    for rank, status, worst, ok in res:
        assert status == "ok", (rank, status)
        assert worst < 1e-5, (rank, worst)
        assert ok, f"rank {rank}: two-shot not used, unaligned not refused, or replicas differ"


def _ddp_overlap_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import torch.nn as nn
    _init(rank, world, port)
    try:
        from raydp_amd.ops import comm as C
        from raydp_amd.parallel.ddp import DistributedDataParallel
        dev = torch.device("cuda", 0)
        g = torch.Generator().manual_seed(21 + rank)
        xs = [torch.randn(128, 64, generator=g).to(dev) for _ in range(5)]
        ys = [torch.randn(128, 1, generator=g).to(dev) for _ in range(5)]
        outs, kinds, launched = {}, {}, {}
        # comm stream + small buckets (several per step) + every xGMI bucket two-shot, against the
        # plain one-bucket stream-ordered one-shot path and the torch.distributed fallback
        cfgs = {"overlap": {"RAYDP_DDP_COMM_STREAM": "1", "RAYDP_ALLREDUCE_TWOSHOT_MIN_MB": "0"},
                "serial": {"RAYDP_DDP_COMM_STREAM": "0", "RAYDP_ALLREDUCE_TWOSHOT_MIN_MB": "1024"},
                "rccl": {"RAYDP_ALLREDUCE": "rccl"}}
        for name, env in cfgs.items():
            os.environ.update(env)
            torch.manual_seed(0)
            net = nn.Sequential(nn.Linear(64, 256), nn.ReLU(), nn.Linear(256, 256), nn.ReLU(),
                                nn.Linear(256, 1)).to(dev)
            ddp = DistributedDataParallel(net, bucket_cap_mb=0.1 if name == "overlap" else None)
            opt = torch.optim.SGD(ddp.parameters(), lr=0.05)
            for x, y in zip(xs, ys):
                ddp.zero_grad()
                nn.functional.mse_loss(ddp(x), y).backward()
                opt.step()
            torch.cuda.synchronize()
            ddp.check_comm()
            outs[name] = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).cpu()
            kinds[name] = (len(ddp.buckets), ddp._allreduce.kind)
            launched[name] = dict(ddp._allreduce.launched)
            for k in env:
                os.environ.pop(k, None)
        gathered = [None] * world
        dist.all_gather_object(gathered, outs["overlap"])
        same = all(bool(torch.equal(gathered[0], t)) for t in gathered)
        q.put((rank, same, float((outs["overlap"] - outs["serial"]).abs().max()),
               float((outs["overlap"] - outs["rccl"]).abs().max()), kinds, launched))
        dist.barrier()
        C.reset_cache()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ddp_buckets_on_comm_stream_twoshot_match_serial(world):
    """Gradient buckets reduced on the comm stream while backward continues (several buckets per
    step, every one two-shot at world > 2) train like the stream-ordered one-shot path and the
    torch.distributed fallback; replicas stay identical."""
    res = _run(_ddp_overlap_main, world)
    for rank, same, d_serial, d_rccl, kinds, launched in res:
        assert same, f"rank {rank}: replicas diverged"
        assert d_serial < 1e-5 and d_rccl < 1e-5, (rank, d_serial, d_rccl)
        assert kinds["overlap"][0] > 1 and "comm_stream" in kinds["overlap"][1], kinds
        if world > 2:
            assert launched["overlap"]["twoshot"] > 0 and launched["serial"]["twoshot"] == 0, launched
        assert launched["rccl"]["oneshot"] == 0 and launched["rccl"]["twoshot"] == 0, launched


def _ddp_error_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import torch.nn as nn
    _init(rank, world, port)
    try:
        from raydp_amd.exceptions import CollectiveError
        from raydp_amd.ops import comm as C
        from raydp_amd.parallel.ddp import DistributedDataParallel
        dev = torch.device("cuda", 0)
        net = nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 1)).to(dev)
        ddp = DistributedDataParallel(net)
        xg = ddp._allreduce.xg
        if rank == 1:
            xg._inject_error()                  # as if rank 1 had missed a peer
        raised = False
        try:
            ddp.check_comm()
        except CollectiveError:
            raised = True
        torch.cuda.synchronize()
        # the rank that retired xGMI and its healthy peers agree on the next set-up: no hang,
        # every rank falls back together
        again = C.XgmiComm.create(1024, timeout_s=5.0, tag="after")
        q.put((rank, raised, ddp._allreduce.xg is None, again is None))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_ddp_xgmi_error_word_raises_and_ranks_fall_back_together():
    """A timed-out exchange on the DDP path is not silent: the epoch-end check raises
    CollectiveError on the rank that saw it, and the next communicator set-up is refused on EVERY
    rank through one agreement collective (no rank left waiting in a different collective)."""
    res = _run(_ddp_error_main, 2)
    assert res[0][1] is False and res[1][1] is True, res
    assert res[1][2], res
    assert all(r[3] for r in res), res
