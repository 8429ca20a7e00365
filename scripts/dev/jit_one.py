import sys, time
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "..", ".."))
import torch, torch.nn as nn
import __graft_entry__ as g
from raydp_amd.ops import mlp_jit
m = g._nyc_model()
t = time.time()
mlp_jit.precompile_many([(m, torch.optim.Adam(m.parameters(), lr=1e-3), nn.SmoothL1Loss(), int(sys.argv[1]) if len(sys.argv) > 1 else 64, None)])
print("ok", time.time() - t)
