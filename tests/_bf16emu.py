"""bf16 operand-rounding emulation of the reference (test infrastructure): the oracle under the rounding C4's kernels
apply, the bar of the C4 parity tests (tests/test_gpu_configs.py) and of the fixture tests/golden/make_golden_r5_c4.py
generates."""
import torch

from oracle import ref_cpu as R


class _RoundBF16(torch.autograd.Function):
    """A tensor stored in bf16 and its gradient stored in bf16 (torch.autocast's conv outputs)."""

    @staticmethod
    def forward(ctx, v):
        return v.to(torch.bfloat16).to(v.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


class _bf16_operands:
    """Oracle hook: round the operands of every 3x3 conv with C_in > 1 and of every ConvTranspose2d (the two k = 2 ones
    and, since round 5 runs its forward on the 16-bit matrix cores, up0's k = h/4) to bf16 (fp32 accumulate), as C4 does
    (the C_in = 1 / C_out = 1 convs stay fp32 on both sides).  outputs=True also
    stores those 3x3 convs' outputs and their gradients in bf16, as torch.autocast does (the HIP C4 train step stores
    the fused chain's y and g in bf16, a subset of these, so this reference is the less precise one)."""

    def __init__(self, outputs: bool = False):
        self.outputs = outputs

    def __enter__(self):
        self.orig, self.orig_t = R.F.conv2d, R.F.conv_transpose2d

        def bf(v):
            return v.to(torch.bfloat16).to(v.dtype)

        def conv(x, w, b=None, *a, **k):
            if w.shape[-1] == 3 and w.shape[1] > 1:
                out = self.orig(bf(x), bf(w), b, *a, **k)
                return _RoundBF16.apply(out) if self.outputs else out
            return self.orig(x, w, b, *a, **k)

        def convt(x, w, b=None, *a, **k):   # both ConvTranspose2d kinds: UnetUp's k = 2 and up0's k = h/4
            return self.orig_t(bf(x), bf(w), b, *a, **k)
        R.F.conv2d, R.F.conv_transpose2d = conv, convt
        return self

    def __exit__(self, *exc):
        R.F.conv2d, R.F.conv_transpose2d = self.orig, self.orig_t
