"""fp8 (OCP e4m3fn) weights: container, quantization and the fp32 reference (BASELINE config 5).

A linear layer's bf16 weight W [rows, K] is stored as W8 (e4m3fn) with one fp32 scale per
row, W ≈ W8 * s[:, None], s = amax|W[row]| / 448. Rows keep their bf16 order, so the packed
gate/up layout and fused qkv rows carry over unchanged. On the GPU:
  * decode (M <= 64)  W8A16 -- weights streamed at 1 byte each, dequantized exactly to bf16
                      in registers (csrc/kernels/gemm_fp8.hip, gemm_fp8_dec);
  * prefill (M > 64)  W8A8  -- activations quantized per token (quant_rows) and multiplied
                      with the block-scaled fp8 MFMA (gemm_fp8_tile).
`reference_linear` reproduces exactly that arithmetic in fp32 (the oracle of the GPU tests and
the CPU path).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import reference as R

FP8 = torch.float8_e4m3fn
FP8_MAX = 448.0
DEC_MAX_M = 64


@dataclass
class Fp8Weight:
    w8: torch.Tensor  # float8_e4m3fn [rows, K]
    scale: torch.Tensor  # fp32 [rows]

    @property
    def shape(self):
        return self.w8.shape

    @property
    def device(self):
        return self.w8.device

    def dequant(self, dtype=torch.float32):
        return (self.w8.float() * self.scale[:, None]).to(dtype)

    def nbytes(self):
        return self.w8.numel() + 4 * self.scale.numel()


def quantize_weight(w: torch.Tensor) -> Fp8Weight:
    """Per-output-row symmetric e4m3fn quantization (round to nearest even, no saturation needed:
    every |w / s| <= 448)."""
    wf = w.float()
    s = wf.abs().amax(dim=1).clamp_min(1e-12) / FP8_MAX
    w8 = (wf / s[:, None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return Fp8Weight(w8.contiguous(), s.contiguous())


def quantize_rows(x: torch.Tensor):
    """Dynamic per-row activation quantization, as the GPU quant_rows kernel does."""
    xf = x.float()
    a = xf.abs().amax(dim=1)
    s = torch.where(a > 0, a * torch.tensor(1.0 / FP8_MAX, dtype=torch.float32), torch.ones_like(a))
    inv = torch.ones_like(s) / s  # correctly rounded, like the kernel's __fdiv_rn
    q = (xf * inv[:, None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return q, s


def reference_linear(x, w: Fp8Weight, bias=None, resid=None, epi="none", out_f32=False):
    """fp32 oracle of ragk_gemm_fp8: W8A16 for M <= 64, W8A8 above."""
    wd = w.dequant()
    if x.shape[0] <= DEC_MAX_M:
        xe = x.float()
    else:
        q, s = quantize_rows(x)
        xe = q.float() * s[:, None]
    y = R.linear(xe, wd, bias, resid, epi=epi, out_f32=True)
    return y if out_f32 else y.to(x.dtype)
