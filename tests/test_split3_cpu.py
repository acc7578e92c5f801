"""The arithmetic of the split-bf16 GEMM (csrc/gemm_split3.hip), checked on the CPU
with torch's bfloat16 conversion (round to nearest even, as v_cvt_pk_bf16_f32):

* the three-piece split x = x0 + x1 + x2 (x0 = bf16(x), x1 = bf16(x - x0),
  x2 = bf16(x - x0 - x1)) leaves a residual <= 2^-24 |x| -- fp32's precision -- over
  fp32 magnitudes from 1e-30 to 1e30;
* the six kept piece products a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 + a2 b0, summed
  exactly (float64), differ from the exact product by <= 2^-22 |a b| (the three
  dropped ones and the split residuals);
* a K = 1024 dot product formed that way and rounded once to fp32 is as close to the
  exact dot product as the correctly rounded fp32 result, up to 2^-20 of sum |a b|.
The GPU kernels' own accumulation is measured against fp64 in
tests/test_gemm_split3_gpu.py."""
import numpy as np
import torch


def split3(x: torch.Tensor):
    x0 = x.to(torch.bfloat16).float()
    r1 = x - x0  # exact in fp32
    x1 = r1.to(torch.bfloat16).float()
    r2 = r1 - x1  # exact in fp32
    x2 = r2.to(torch.bfloat16).float()
    return x0, x1, x2


def test_split_residual_within_fp32_precision():
    g = torch.Generator().manual_seed(0)
    mags = torch.logspace(-30, 30, 61)
    x = (torch.randn(61, 4096, generator=g) * mags[:, None]).float().flatten()
    x0, x1, x2 = split3(x)
    # the pieces are bf16 values and the sum of the first two is exact in fp32
    for p in (x0, x1, x2):
        assert torch.equal(p, p.to(torch.bfloat16).float())
    res = (x.double() - (x0.double() + x1.double() + x2.double())).abs()
    assert bool((res <= 2.0 ** -24 * x.double().abs()).all()), float((res / x.abs()).max())
    # the pieces shrink by ~2^-8 each
    nz = x != 0
    assert bool((x1.abs() <= 2.0 ** -8 * x.abs())[nz].all())
    assert bool((x2.abs() <= 2.0 ** -16 * x.abs())[nz].all())


def test_six_products_within_2e22():
    g = torch.Generator().manual_seed(1)
    a = torch.randn(1 << 16, generator=g) * 3
    b = torch.randn(1 << 16, generator=g) * 0.05
    a0, a1, a2 = (p.double() for p in split3(a))
    b0, b1, b2 = (p.double() for p in split3(b))
    six = a0 * b0 + a0 * b1 + a1 * b0 + a0 * b2 + a1 * b1 + a2 * b0
    exact = a.double() * b.double()
    err = (six - exact).abs()
    assert bool((err <= 2.0 ** -22 * exact.abs()).all()), float((err / exact.abs()).max())


def test_dot_product_as_accurate_as_fp32_rounding():
    g = torch.Generator().manual_seed(2)
    K = 1024
    a = torch.randn(256, K, generator=g)
    b = torch.randn(K, generator=g) / K ** .5
    A = [p.double() for p in split3(a)]
    B = [p.double() for p in split3(b)]
    six = (A[0] @ B[0] + A[0] @ B[1] + A[1] @ B[0] + A[0] @ B[2] + A[1] @ B[1] + A[2] @ B[0])
    exact = a.double() @ b.double()
    scale = (a.double().abs() @ b.double().abs())
    e_six = (six.float().double() - exact).abs()
    e_fp32 = (exact.float().double() - exact).abs()  # one correct rounding
    assert bool((e_six <= e_fp32 + 2.0 ** -20 * scale).all())
    assert float(np.mean((e_six / scale).numpy())) < 1e-7
