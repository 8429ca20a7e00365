"""Host-side decisions of the fused optimizers (no GPU needed)."""
import torch

from raydp_amd.ops.fused_optim import sgd_supported


def test_sparse_gradient_with_momentum_goes_to_torch():
    # torch.optim.SGD keeps a (densified) momentum buffer for sparse gradients; the fused step
    # only implements plain SGD for them, so it must decline
    emb = torch.nn.Embedding(10, 4, sparse=True)
    emb(torch.tensor([1, 3])).sum().backward()
    assert emb.weight.grad.is_sparse
    assert sgd_supported(torch.optim.SGD(emb.parameters(), lr=0.1, momentum=0.9)) == "sparse gradient with momentum"
    assert sgd_supported(torch.optim.SGD(emb.parameters(), lr=0.1)) is None
