"""The GEMM epilogues' GELU / GELU' lookup tables (vjepa2_amd/gelu_tables.py) against PyTorch's own
fp32 GELU on every bf16 input (CPU, no GPU needed). The device lookup (gelu_tab_bf16 /
gelu_grad_tab in vj_gemm256.hip) is emulated here entry for entry."""
import numpy as np
import torch

from vjepa2_amd import gelu_tables as gt


def _lookup_fwd(bits, fwd):
    e = (bits >> 7) & 0xFF
    rel = e.astype(np.int64) - gt.E_LO
    inr = (rel >= 0) & (rel < gt.NEXP)
    idx = np.where(inr, (bits >> 15) * (gt.NEXP * 128) + rel * 128 + (bits & 127), 0)
    x = (bits.astype(np.uint32) << 16).view(np.float32)
    with np.errstate(invalid="ignore"):
        xh = x * np.float32(0.5)
    half = torch.from_numpy(xh).bfloat16().view(torch.int16).numpy().astype(np.uint16)
    big = np.where(bits & 0x8000, np.uint16(0x8000), bits.astype(np.uint16))
    return np.where(inr, fwd[idx], np.where(e < gt.E_LO, half, big))


def test_gelu_table_matches_torch_fp32_gelu():
    fwd, bwd = gt.build_tables()
    bits = np.arange(65536, dtype=np.int64)
    x = torch.from_numpy((bits.astype(np.uint32) << 16).view(np.float32))
    finite = (x.abs() < 1e30).numpy()  # torch overflows x*(1+erf) near fp32 max; the table keeps x
    ours = _lookup_fwd(bits, fwd)[finite]
    ref = torch.nn.functional.gelu(x).bfloat16().view(torch.int16).numpy().astype(np.uint16)[finite]
    same = (ours == ref) | (((ours & 0x7FFF) == 0) & ((ref & 0x7FFF) == 0))  # +-0 alike
    # Only where 1 + erf(x/sqrt2) cancels (x < -3) can torch's vectorised CPU erf (not correctly
    # rounded) move the fp32 result across a bf16 rounding boundary: there, at most 2 bf16 ulps.
    # (there the result is ~1e-3..1e-7 with few significant bits: compare absolutely)
    xs = x.numpy()[finite]
    assert bool((xs[~same] < -3).all())
    to_f = lambda u: (u.astype(np.uint32) << 16).view(np.float32)  # noqa: E731
    assert float(np.abs(to_f(ours[~same]) - to_f(ref[~same])).max(initial=0)) <= 2e-5


def test_gelu_grad_table_matches_torch():
    fwd, bwd = gt.build_tables()
    ins = np.array(gt.table_inputs(), dtype=np.uint32)
    x = torch.from_numpy((ins << 16).view(np.float32)).requires_grad_(True)
    torch.nn.functional.gelu(x).backward(torch.ones_like(x))
    ref = x.grad.numpy()
    # cdf + x*pdf cancels for x < 0: the two fp32 evaluations may differ by an ulp of the O(1) terms
    np.testing.assert_allclose(bwd, ref, rtol=2e-6, atol=2.4e-7)
