"""bin_sums_kernel (csrc/binsum.hip) vs the fp64 index_add_ reference."""
import pytest
import torch

from orange3_spark_amd.ops import binsum as BS


def test_cpu_bin_sums_layout():
    X = torch.tensor([[1.0, 2.0], [3.0, 4.0], [5.0, 6.0]])
    b = torch.tensor([1, -1, 1])
    out = BS.bin_sums(X, b, 2)
    assert out.shape == (2, 4)
    assert out[1].tolist() == [6.0, 8.0, 2.0, 1 + 4 + 25 + 36]
    assert out[0].tolist() == [0.0, 0.0, 0.0, 0.0]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,D,nbins,weighted", [(torch.float32, 64, 16, False), (torch.bfloat16, 130, 5, True),
                                                    (torch.float64, 3, 300, True), (torch.float32, 256, 9, False)])
def test_gpu_bin_sums_matches_index_add(gpu, dtype, D, nbins, weighted):
    g = torch.Generator().manual_seed(D + nbins)
    n = 300_001
    X = (torch.randn((n, D), generator=g)).to(dtype).to(gpu)
    b = torch.randint(-2, nbins + 2, (n,), generator=g).to(gpu)      # out-of-range rows are ignored
    w = (torch.rand(n, generator=g) + 0.5).to(gpu) if weighted else None
    got = BS.bin_sums(X, b, nbins, w)
    ref = BS.bin_sums_torch(X, b, nbins, None if w is None else w.float())
    assert torch.allclose(got, ref, rtol=1e-9, atol=1e-7 * n)
    again = BS.bin_sums(X, b, nbins, w)
    assert torch.equal(got, again)                                   # deterministic
