"""The Horovod NYC user loop (bench.py hvd_train_fn) in ONE process on the GPU, with the
graph_user_model policy applied to the module through hvd.DistributedOptimizer, under the worker
policies (native BatchNorm), printing progress per step: finds where a capture goes wrong.

  RAYDP_GRAPH_HVD_MODEL=1 python -X faulthandler scripts/dev/hvd_graph_repro.py [--no-native-bn]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.nn.functional as F
    import bench
    import raydp_amd.hvd as hvd
    from raydp_amd.train.gpu_policy import worker_policies
    native = "--no-native-bn" not in sys.argv
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator().manual_seed(0)
    X = torch.randn(64 * 40, 20, generator=g).to(dev)
    Y = torch.randn(64 * 40, 1, generator=g).to(dev)
    ctx = worker_policies(True) if native else __import__("contextlib").nullcontext()
    with ctx:
        hvd.init()
        torch.manual_seed(0)
        model = bench.nyc_model(20).to(dev)
        opt = torch.optim.Adam(model.parameters(), lr=0.01)
        hvd.broadcast_parameters(model.state_dict(), root_rank=0)
        hvd.broadcast_optimizer_state(opt, root_rank=0)
        opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(), op=hvd.Average)
        print("graphed:", getattr(model, "_raydp_graphed", False), "native_bn:", native, flush=True)
        t0 = time.perf_counter()
        for ep in range(3):
            model.train()
            for i in range(40):
                opt.zero_grad()
                loss = F.smooth_l1_loss(model(X[i * 64:(i + 1) * 64]), Y[i * 64:(i + 1) * 64])
                loss.backward()
                opt.step()
                if i % 10 == 0:
                    print(f"epoch {ep} step {i} loss {loss.item():.4f}", flush=True)
            torch.cuda.synchronize()
            print(f"epoch {ep}: {(time.perf_counter() - t0) * 1e3:.1f} ms total", flush=True)


if __name__ == "__main__":
    main()
