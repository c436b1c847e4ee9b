"""GPU parity of the training path (bf16 HIP kernels through the C ABI).

Tolerances (bf16 activations, f32 accumulation and master weights):
  * attention backward vs torch fp32 autograd on the same bf16 inputs: max abs error
    <= 2e-2 * max |reference gradient| per tensor (dQ, dK, dV);
  * Linear backward: relative Frobenius error <= 1e-2;
  * focal loss kernel vs the numpy oracle (pinned by the reference's autograd values in
    tests/golden/focal.npz): 1e-5 relative;
  * fused Adam + clip vs the numpy oracle: 1e-5 relative;
  * whole-model gradients vs the REFERENCE model's autograd (tests/golden/train_tiny.npz,
    train mode, dropout 0): per parameter relative Frobenius error <= 8e-2 and cosine
    >= 0.99 for every parameter whose reference gradient norm is non-negligible (measured:
    2-3 % / 0.9996 on the encoder, fusion and head weights), except the AF Fourier
    frequencies (0.15) and the PositionFeatModule convolutions/BatchNorms behind two
    batch-statistic BatchNorms (0.5 / cos 0.85: the BN backward cancellation amplifies the
    bf16 noise of their incoming gradient); loss within 1e-2 relative.
"""

import math

import numpy as np
import pytest
import torch

from conftest import golden_state_dict, load_golden
from oracle import train_np

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _attn_ref(qkv, nseq, L, H, dh):
    D = H * dh
    x = qkv.view(nseq, L, 3, H, dh).permute(2, 0, 3, 1, 4)
    q, k, v = x[0], x[1], x[2]
    p = torch.softmax((q @ k.transpose(-1, -2)) / math.sqrt(dh), -1)
    return (p @ v).permute(0, 2, 1, 3).reshape(nseq * L, D)


@pytest.mark.parametrize("nseq,L,H,dh", [(2, 1030, 2, 32), (3, 200, 3, 64), (1, 77, 1, 32)])
def test_attention_backward_vs_torch(nseq, L, H, dh):
    from src import kernels as K
    g = torch.Generator(device="cpu").manual_seed(L + dh)
    D = H * dh
    qkv = (torch.randn(nseq * L, 3 * D, generator=g) * 1.5).to(DEV, torch.bfloat16)
    dout = torch.randn(nseq * L, D, generator=g).to(DEV, torch.bfloat16)
    out, lse = K.attention_train_fwd(qkv, nseq, L, H, dh)
    ref_in = qkv.float().clone().requires_grad_(True)
    ref = _attn_ref(ref_in, nseq, L, H, dh)
    torch.testing.assert_close(out.float(), ref.detach(), rtol=2e-2, atol=2e-2)
    ref.backward(dout.float())
    got = K.attention_bwd(qkv, out, dout, lse, nseq, L, H, dh).float()
    for i, name in enumerate("qkv"):
        a = got[:, i * D:(i + 1) * D]
        b = ref_in.grad[:, i * D:(i + 1) * D]
        err = (a - b).abs().max().item()
        assert err <= 2e-2 * b.abs().max().item() + 1e-3, (name, err, b.abs().max().item())


@pytest.mark.parametrize("nseq,L,H,dh,p", [(2, 1030, 2, 32, 0.1), (1, 200, 3, 64, 0.3)])
def test_attention_dropout_forward_backward_vs_torch(nseq, L, H, dh, p):
    """Attention-probability dropout (attention.py:28-29): the HIP forward/backward with the
    counter-based keep mask vs torch autograd of softmax(...) * mask / (1 - p) @ V with the same
    mask (tests/attn_helpers.py restates the hash); keep rate ~ 1 - p; the seed changes the mask."""
    from src import kernels as K
    from attn_helpers import keep_mask
    g = torch.Generator(device="cpu").manual_seed(L + 7)
    D = H * dh
    qkv = (torch.randn(nseq * L, 3 * D, generator=g) * 0.8).to(DEV, torch.bfloat16)
    dout = torch.randn(nseq * L, D, generator=g).to(DEV, torch.bfloat16)
    seed = 0x1234567890ABCDEF
    keep = torch.from_numpy(keep_mask(seed, nseq, H, L, p)).to(DEV)
    assert abs(keep.float().mean().item() - (1 - p)) < 0.01
    assert (torch.from_numpy(keep_mask(seed + 1, nseq, H, L, p)).to(DEV) != keep).float().mean() > 0.05
    # the two keys of a hash pair (16-bit halves of one hash) drop independently
    kp = keep.view(nseq, H, L, L // 2, 2)
    assert abs((~kp[..., 0] & ~kp[..., 1]).float().mean().item() - p * p) < 0.01
    out, lse = K.attention_train_fwd(qkv, nseq, L, H, dh, p, seed)
    ref_in = qkv.float().clone().requires_grad_(True)
    x = ref_in.view(nseq, L, 3, H, dh).permute(2, 0, 3, 1, 4)
    P = torch.softmax((x[0] @ x[1].transpose(-1, -2)) / math.sqrt(dh), -1)
    ref = ((P * keep / (1 - p)) @ x[2]).permute(0, 2, 1, 3).reshape(nseq * L, D)
    torch.testing.assert_close(out.float(), ref.detach(), rtol=2e-2, atol=2e-2)
    ref.backward(dout.float())
    got = K.attention_bwd(qkv, out, dout, lse, nseq, L, H, dh, p, seed).float()
    for i, name in enumerate("qkv"):
        a = got[:, i * D:(i + 1) * D]
        b = ref_in.grad[:, i * D:(i + 1) * D]
        err = (a - b).abs().max().item()
        assert err <= 2e-2 * b.abs().max().item() + 1e-3, (name, err, b.abs().max().item())


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_train_overflow_fallback_with_dropout(p):
    """Scores far above the first key tile's max overflow the fixed shift of the training
    forward too: the online-max fallback must apply the same (pair-hash) keep mask and return
    the same lse, so forward and backward still match torch.  (The softmax is saturated here,
    so dQ is tiny next to the bf16 rounding of its O(1) terms: gradients are held to 2 % of the
    largest gradient of the three.)"""
    from src import kernels as K
    from attn_helpers import keep_mask
    nseq, L, H, dh = 2, 300, 2, 32
    g = torch.Generator(device="cpu").manual_seed(5)
    D = H * dh
    qkv = torch.randn(nseq * L, 3 * D, generator=g) * 0.1
    qkv[:, :D] = 4.0
    qkv[200, D:2 * D] = 8.0
    qkv = qkv.to(DEV, torch.bfloat16)
    dout = torch.randn(nseq * L, D, generator=g).to(DEV, torch.bfloat16)
    seed = 0x0BADC0FFEE
    keep = torch.from_numpy(keep_mask(seed, nseq, H, L, p)).to(DEV) if p > 0 else torch.ones(
        nseq, H, L, L, dtype=torch.bool, device=DEV)
    K.attention_fallbacks(True)
    out, lse = K.attention_train_fwd(qkv, nseq, L, H, dh, p, seed)
    assert K.attention_fallbacks(True) > 0
    ref_in = qkv.float().clone().requires_grad_(True)
    x = ref_in.view(nseq, L, 3, H, dh).permute(2, 0, 3, 1, 4)
    s_ = (x[0] @ x[1].transpose(-1, -2)) / math.sqrt(dh)
    P = torch.softmax(s_, -1)
    ref = ((P * keep / (1 - p)) @ x[2]).permute(0, 2, 1, 3).reshape(nseq * L, D)
    assert torch.isfinite(out.float()).all()
    torch.testing.assert_close(out.float(), ref.detach(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(lse, (torch.logsumexp(s_, -1) / math.log(2.0)).detach(), rtol=1e-3, atol=2e-2)
    ref.backward(dout.float())
    got = K.attention_bwd(qkv, out, dout, lse, nseq, L, H, dh, p, seed).float()
    scale = ref_in.grad.abs().max().item()
    for i, name in enumerate("qkv"):
        a = got[:, i * D:(i + 1) * D]
        b = ref_in.grad[:, i * D:(i + 1) * D]
        err = (a - b).abs().max().item()
        assert err <= 2e-2 * scale + 1e-3, (name, err, scale)


def test_attention_lse_matches_logsumexp():
    from src import kernels as K
    nseq, L, H, dh = 2, 300, 2, 32
    qkv = torch.randn(nseq * L, 3 * H * dh, device=DEV).to(torch.bfloat16)
    _, lse = K.attention_train_fwd(qkv, nseq, L, H, dh)
    x = qkv.float().view(nseq, L, 3, H, dh).permute(2, 0, 3, 1, 4)
    s = (x[0] @ x[1].transpose(-1, -2)) / math.sqrt(dh)
    ref = torch.logsumexp(s, -1) / math.log(2.0)
    torch.testing.assert_close(lse, ref, rtol=1e-3, atol=2e-2)


@pytest.mark.parametrize("M,K_,N,multi", [(1000, 384, 1152, True), (777, 64, 384, False), (512, 1536, 384, False)])
def test_hip_linear_backward(M, K_, N, multi):
    from src.autograd_ops import hip_linear
    g = torch.Generator(device="cpu").manual_seed(M)
    x = torch.randn(M, K_, generator=g).to(DEV, torch.bfloat16).requires_grad_(True)
    if multi:
        ws = [(torch.randn(N // 3, K_, generator=g) / math.sqrt(K_)).to(DEV).requires_grad_(True) for _ in range(3)]
        bs = [torch.randn(N // 3, generator=g).to(DEV).requires_grad_(True) for _ in range(3)]
    else:
        ws = [(torch.randn(N, K_, generator=g) / math.sqrt(K_)).to(DEV).requires_grad_(True)]
        bs = [torch.randn(N, generator=g).to(DEV).requires_grad_(True)]
    gy = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    y = hip_linear(x, ws if multi else ws[0], bs if multi else bs[0])
    y.backward(gy)
    xr = x.detach().float().requires_grad_(True)
    wr = [w.detach().to(torch.bfloat16).float().requires_grad_(True) for w in ws]
    br = [b.detach().clone().requires_grad_(True) for b in bs]
    yr = xr @ torch.cat(wr).t() + torch.cat(br)
    yr.backward(gy.float())
    rel = lambda a, b: ((a.float() - b).norm() / b.norm()).item()
    assert rel(y, yr.detach()) < 1e-2
    assert rel(x.grad, xr.grad) < 1e-2
    for w, r in zip(ws, wr):
        assert rel(w.grad, r.grad) < 1e-2
    for b, r in zip(bs, br):
        assert rel(b.grad, r.grad) < 1e-2


@pytest.mark.parametrize("M,N,K_,splits", [(1, 128, 128, 0), (1000, 1152, 384, 0), (4097, 384, 1536, 0),
                                            (4097, 384, 1536, 3), (24 * 2 * 1025, 384, 384, 0), (33, 256, 128, 64)])
def test_linear_dw_kernel_vs_fp32(M, N, K_, splits):
    """dW = dy^T x and db = sum dy (csrc/dw.hip) against fp32 torch on the same bf16 values: ragged
    M (not a multiple of the 32-row stage), more chunks than stages, the bench's 2BL rows."""
    from src import kernels as K
    g = torch.Generator(device="cpu").manual_seed(M + N)
    dy = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    x = torch.randn(M, K_, generator=g).to(DEV, torch.bfloat16)
    dw, db = K.linear_dw(dy, x, bias=True, splits=splits)
    ref_w = dy.double().t() @ x.double()
    ref_b = dy.double().sum(0)
    tol = 1e-5 * math.sqrt(M) * 4
    assert (dw.double() - ref_w).abs().max().item() < tol
    assert (db.double() - ref_b).abs().max().item() < tol
    dw2, none = K.linear_dw(dy, x)
    assert none is None and (dw2.double() - ref_w).abs().max().item() < tol
    if N % 384 == 0:
        # one launch over three equal parts with separate (accumulated) output buffers
        parts_w = [torch.ones(N // 3, K_, device=DEV) for _ in range(3)]
        parts_b = [torch.ones(N // 3, device=DEV) for _ in range(3)]
        K.linear_dw_parts(dy, x, parts_w, parts_b)
        assert (torch.cat(parts_w).double() - 1 - ref_w).abs().max().item() < tol
        assert (torch.cat(parts_b).double() - 1 - ref_b).abs().max().item() < tol
    if N % 256 == 0:
        # a column slice of dy (strided rows), accumulated onto existing values (a .grad buffer)
        h = N // 2
        acc_w = torch.randn(N - h, K_, generator=g).to(DEV)
        acc_b = torch.randn(N - h, generator=g).to(DEV)
        want_w = acc_w.double() + ref_w[h:]
        want_b = acc_b.double() + ref_b[h:]
        K.linear_dw(dy[:, h:], x, dw=acc_w, db=acc_b, splits=splits)
        assert (acc_w.double() - want_w).abs().max().item() < tol
        assert (acc_b.double() - want_b).abs().max().item() < tol


@pytest.mark.parametrize("p_r,p_out", [(0.1, 0.19), (0.0, 0.1), (0.3, 0.0)])
def test_layernorm_fused_dropout_vs_torch(p_r, p_out):
    """drop_o(LN(x + drop_r(r))) with the masks fused into the LN kernels (csrc/train.hip) ==
    torch on the same masks (tests/attn_helpers.py restates the hash): output, dx, dr, dg, db;
    with direct_weight_grads the LN parameter gradients land in their .grad buffers (added)."""
    from attn_helpers import ln_keep_mask
    from src import autograd_ops as A
    from src import kernels as K
    M, N = 1031, 384
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16).requires_grad_(True)
    r = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16).requires_grad_(True)
    ln = torch.nn.LayerNorm(N).to(DEV)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.5, 0.5)
    seed = 0x1234_5678_9ABC
    gy = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    y = A._HipAddLayerNorm.apply(x, r, ln.weight, ln.bias, ln.eps, p_r, p_out, seed)
    y.backward(gy)
    mr = torch.from_numpy(ln_keep_mask(seed, 0, M, N, p_r)).to(DEV).float() / (1 - p_r)
    mo = torch.from_numpy(ln_keep_mask(seed, 1, M, N, p_out)).to(DEV).float() / (1 - p_out)
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True)
    lr = torch.nn.LayerNorm(N).to(DEV)
    lr.load_state_dict(ln.state_dict())
    s = (xr + rr * mr).to(torch.bfloat16).float()          # the kernel keeps s in bf16
    yr = lr(s) * mo
    yr.backward(gy.float())
    rel = lambda a, b: ((a.float() - b).norm() / b.norm()).item()
    assert rel(y, yr.detach()) < 1e-2
    assert rel(x.grad, xr.grad) < 2e-2 and rel(r.grad, rr.grad) < 2e-2
    assert rel(ln.weight.grad, lr.weight.grad) < 1e-2 and rel(ln.bias.grad, lr.bias.grad) < 1e-2
    # direct accumulation into the parameters' .grad
    w0, b0 = ln.weight.grad.clone(), ln.bias.grad.clone()
    with A.direct_weight_grads():
        A._HipAddLayerNorm.apply(x, r, ln.weight, ln.bias, ln.eps, p_r, p_out, seed).backward(gy)
    torch.testing.assert_close(ln.weight.grad, 2 * w0, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(ln.bias.grad, 2 * b0, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,N,resid", [(1000, 384, True), (517, 1536, False), (64, 64, True)])
def test_hip_add_layernorm_fwd_bwd(M, N, resid):
    from src.autograd_ops import hip_add_layernorm
    g = torch.Generator(device="cpu").manual_seed(N)
    ln = torch.nn.LayerNorm(N).to(DEV)
    with torch.no_grad():
        ln.weight.copy_(torch.randn(N, generator=g) * 0.5 + 1)
        ln.bias.copy_(torch.randn(N, generator=g) * 0.1)
    x = (torch.randn(M, N, generator=g) * 3 + 1).to(DEV, torch.bfloat16).requires_grad_(True)
    r = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16).requires_grad_(True) if resid else None
    gy = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    y = hip_add_layernorm(x, r, ln)
    y.backward(gy)
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if resid else None
    s = (xr + rr).bfloat16().float() if resid else xr          # the kernel keeps x + r in bf16
    wr, br = ln.weight.detach().clone().requires_grad_(True), ln.bias.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(s, (N,), wr, br, ln.eps)
    yr.backward(gy.float())
    rel = lambda a, b: ((a.float() - b).norm() / b.norm()).item()
    assert rel(y, yr.detach()) < 1e-2
    assert rel(x.grad, xr.grad) < 1e-2
    if resid:
        assert rel(r.grad, rr.grad) < 1e-2
    assert rel(ln.weight.grad, wr.grad) < 1e-3 and rel(ln.bias.grad, br.grad) < 1e-3


@pytest.mark.parametrize("M,N,mode", [(300, 1536, "x"), (257, 384, "r"), (64, 384, "r_drop")])
def test_hip_add_layernorm_fused_leaky_relu(M, N, mode):
    """FeedForward's LeakyReLUs fused into the LayerNorm kernels (feed_forward.py:20-21): mode x:
    y = LN(lrelu(x)) (the FFN norm on w_1's pre-activation output); r: y = LN(x + lrelu(r)) (the
    output sublayer on w_2's pre-activation output); r_drop: the same with residual dropout
    (checked against the un-fused kernel path on identical masks: same seed).  Forward and every
    gradient vs torch f32 autograd on the same bf16 inputs, 1e-2 relative (bf16 outputs)."""
    from src.autograd_ops import hip_add_layernorm
    import src.autograd_ops as A
    g = torch.Generator(device="cpu").manual_seed(N + M)
    ln = torch.nn.LayerNorm(N).to(DEV)
    with torch.no_grad():
        ln.weight.copy_(torch.randn(N, generator=g) * 0.5 + 1)
        ln.bias.copy_(torch.randn(N, generator=g) * 0.1)
    x = (torch.randn(M, N, generator=g) * 2).to(DEV, torch.bfloat16).requires_grad_(True)
    r = (torch.randn(M, N, generator=g) * 2).to(DEV, torch.bfloat16).requires_grad_(True)
    gy = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()
    if mode == "r_drop":
        seed = 1234
        orig = A._drop_seed
        A._drop_seed = lambda: seed
        try:
            y = hip_add_layernorm(x, r, ln, p_r=0.2, act_r=0.1)
            y.backward(gy)
            gx, gr, gw = x.grad.clone(), r.grad.clone(), ln.weight.grad.clone()
            x.grad = r.grad = None
            ln.weight.grad = ln.bias.grad = None
            ra = torch.nn.functional.leaky_relu(r, 0.1)            # the un-fused path, same seed
            y2 = hip_add_layernorm(x, ra, ln, p_r=0.2)
            y2.backward(gy)
        finally:
            A._drop_seed = orig
        assert rel(y, y2) < 1e-3 and rel(gx, x.grad) < 1e-3 and rel(gr, r.grad) < 1e-2 and rel(gw, ln.weight.grad) < 1e-3
        return
    y = hip_add_layernorm(x, None, ln, act_x=0.1) if mode == "x" else hip_add_layernorm(x, r, ln, act_r=0.1)
    y.backward(gy)
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True)
    wr, br = ln.weight.detach().clone().requires_grad_(True), ln.bias.detach().clone().requires_grad_(True)
    if mode == "x":
        s = torch.nn.functional.leaky_relu(xr, 0.1)
    else:
        s = xr + torch.nn.functional.leaky_relu(rr, 0.1)
    yr = torch.nn.functional.layer_norm(s, (N,), wr, br, ln.eps)
    yr.backward(gy.float())
    assert rel(y, yr.detach()) < 1e-2
    assert rel(x.grad, xr.grad) < 1e-2
    if mode == "r":
        assert rel(r.grad, rr.grad) < 1e-2
    assert rel(ln.weight.grad, wr.grad) < 2e-3 and rel(ln.bias.grad, br.grad) < 2e-3


@pytest.mark.parametrize("N", [384, 1536])
def test_hip_linear_rank2_vs_torch(N):
    """Linear(cat([x, c1, c2])) with the two extra columns as stream-GEMM epilogue rank terms
    (fusion.py:355-360, the hap head's af_fusion[0]): output and the gradients of x, c1, c2, W and
    b vs torch f32 autograd of the concatenated form on the same bf16-rounded operands, 1e-2
    relative (bf16 output and bf16 dz)."""
    from src.autograd_ops import hip_linear_rank2
    g = torch.Generator(device="cpu").manual_seed(N)
    M, D = 2 * 1030 + 6, 384
    lin = torch.nn.Linear(D + 2, N).to(DEV)
    x = (torch.randn(M, D, generator=g)).to(DEV, torch.bfloat16).requires_grad_(True)
    c1 = torch.randn(M, generator=g).to(DEV).requires_grad_(True)
    c2 = torch.rand(M, generator=g).to(DEV).requires_grad_(True)
    gz = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    z = hip_linear_rank2(x, lin, c1, c2)
    assert z.dtype == torch.bfloat16
    z.backward(gz)
    xr = x.detach().float().requires_grad_(True)
    c1r, c2r = c1.detach().clone().requires_grad_(True), c2.detach().clone().requires_grad_(True)
    Wr = lin.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    br = lin.bias.detach().clone().requires_grad_(True)
    zr = torch.nn.functional.linear(torch.cat([xr, c1r[:, None], c2r[:, None]], -1), Wr, br)
    zr.backward(gz.float())
    rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()
    assert rel(z, zr.detach()) < 1e-2
    assert rel(x.grad, xr.grad) < 1e-2
    assert rel(c1.grad, c1r.grad) < 1e-2 and rel(c2.grad, c2r.grad) < 1e-2
    assert rel(lin.weight.grad, Wr.grad) < 1e-2 and rel(lin.bias.grad, br.grad) < 1e-2


def test_fused_neighbour_mean_dropout_vs_torch():
    """K.nbr_mean_drop (train-mode neighbour K-mean, one dropout mask per unique neighbour,
    embedding_rag_dataset.py:404-417): p = 0 equals the torch form (embed the unique neighbours,
    average per query) at 1e-5; with p = 0.3 the kept fraction is 0.7 and the mean is unbiased, and
    the backward is the exact adjoint of the (linear in W, Ar) forward under the same mask:
    <f(W + dW, Ar + dA) - f(W, Ar), R> = <gW(R), dW> + <gAr(R), dA>."""
    from src import kernels as K
    g = torch.Generator(device="cpu").manual_seed(11)
    nq, k, U, L, D, n = 12, 8, 40, 300, 64, 290
    inv = torch.randint(0, U, (nq, k), generator=g).to(torch.int32)
    inv[3, 5:] = -1
    codes = torch.randint(0, 2, (U, n), generator=g).to(torch.uint8)
    W = torch.randn(10, D, generator=g)
    W[0] = 0
    pe = torch.randn(L, D, generator=g) * 0.1
    Ar = torch.randn(L, D, generator=g) * 0.1
    d = lambda t: t.to(DEV)
    # torch reference at p = 0
    tok = torch.zeros(U, L, dtype=torch.long)
    tok[:, 0] = 2
    tok[:, n + 1] = 3
    tok[:, 1:1 + n] = 5 + codes.long()
    E = W[tok] + pe + Ar                                   # [U, L, D]
    ref = torch.stack([E[inv[q][inv[q] >= 0].long()].mean(0) for q in range(nq)])
    out0 = K.nbr_mean_drop(d(inv), d(codes), n, d(W), d(pe), d(Ar), 0.0, 1)
    torch.testing.assert_close(out0.cpu(), ref, rtol=1e-5, atol=1e-5)
    # dropout: keep rate and unbiasedness (each element is kept-and-scaled or 0)
    p = 0.3
    outs = torch.stack([K.nbr_mean_drop(d(inv), d(codes), n, d(W), d(pe), d(Ar), p, s) for s in range(24)])
    assert abs((outs.mean(0).cpu() - ref).abs().mean().item()) < 0.1 * ref.abs().mean().item()
    one = K.nbr_mean_drop(d(inv[:, :1].contiguous()), d(codes), n, d(W), d(pe), d(Ar), p, 5).cpu()
    base = E[inv[:, 0].long()]
    kept = (one != 0) & (base != 0)
    assert abs(kept.float().sum().item() / (base != 0).sum().item() - (1 - p)) < 0.01
    torch.testing.assert_close(one[kept], (base / (1 - p))[kept], rtol=1e-5, atol=1e-5)
    # adjoint identity under one fixed mask
    R = torch.randn(nq, L, D, generator=g)
    dW0 = torch.randn(10, D, generator=g) * 0.01
    dA0 = torch.randn(L, D, generator=g) * 0.01
    f0 = K.nbr_mean_drop(d(inv), d(codes), n, d(W), d(pe), d(Ar), p, 9).cpu().double()
    f1 = K.nbr_mean_drop(d(inv), d(codes), n, d(W + dW0), d(pe), d(Ar + dA0), p, 9).cpu().double()
    gW = torch.zeros(10, D, device=DEV)
    gA = torch.zeros(L, D, device=DEV)
    K.nbr_mean_drop_bwd(d(R), d(inv), d(codes), n, d(W), d(pe), d(Ar), p, 9, gW, gA)
    gW = gW.cpu().double()
    gW[0] = 0                                              # <pad>: no gradient (padding_idx)
    dW_nopad = dW0.double().clone()
    dW_nopad[0] = 0
    lhs = ((f1 - f0) * R.double()).sum().item()
    rhs = (gW * dW_nopad).sum().item() + (gA.cpu().double() * dA0.double()).sum().item()
    # the <pad> row enters the forward (W[0]) but gets no gradient: exclude its contribution
    pad_part = K.nbr_mean_drop(d(inv), d(codes), n, d(W + torch.cat([dW0[:1], torch.zeros(9, D)])), d(pe),
                               d(Ar), p, 9).cpu().double()
    lhs -= ((pad_part - f0) * R.double()).sum().item()
    assert abs(lhs - rhs) < 1e-4 * max(1.0, abs(rhs)), (lhs, rhs)


def test_focal_loss_kernel_vs_oracle_and_reference():
    from src import kernels as K
    z = load_golden("focal")
    for C in (2, 4):
        x, y, m = z[f"x{C}"], z[f"y{C}"], z[f"m{C}"]
        loss, grad = K.focal_loss(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV),
                                  torch.from_numpy(m).to(DEV), 2.0, 1.0)
        np.testing.assert_allclose(loss.item(), float(z[f"loss{C}"]), rtol=1e-5)
        np.testing.assert_allclose(grad.cpu().numpy(), z[f"grad{C}"], rtol=1e-4, atol=1e-6)
        ol, og = train_np.focal_loss(x, y, m)
        np.testing.assert_allclose(loss.item(), ol, rtol=1e-5)


def test_fused_adam_with_clip_vs_oracle():
    from src.main.optimizer import FlatParams, FusedAdam
    g = torch.Generator(device="cpu").manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(s, generator=g).to(DEV)) for s in ((37, 5), (64,), (3, 3, 7))]
    fp = FlatParams(params)
    opt = FusedAdam(fp, lr=1e-2, betas=(0.9, 0.98), eps=1e-8, weight_decay=0.01, max_grad_norm=1.0)
    p0 = fp.flat.cpu().numpy().copy()
    m = np.zeros_like(p0)
    v = np.zeros_like(p0)
    for step in range(1, 4):
        for p in params:
            p.grad.copy_(torch.randn(p.shape, generator=g).to(DEV) * 3)
        gr = fp.grad.cpu().numpy().copy()
        opt.step(grad_scale=0.5)
        p0, m, v = train_np.adam_step(p0, gr, m, v, lr=1e-2, betas=(0.9, 0.98), eps=1e-8, weight_decay=0.01,
                                      step=step, grad_scale=0.5, max_norm=1.0)
        np.testing.assert_allclose(fp.flat.cpu().numpy(), p0, rtol=1e-5, atol=1e-6)
    # the bf16 mirror the GEMMs read follows the update
    np.testing.assert_allclose(fp.bf16.float().cpu().numpy(), p0, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("n", [1, 7, 4096 + 3, 26_000_001])
def test_sqnorm_deterministic_and_exact(n):
    """The clip norm every data-parallel rank derives from the same reduced gradient must agree
    bit for bit (fixed-order two-pass sum), and match float64 to f32 summation accuracy."""
    from src import kernels as K
    x = torch.randn(n, generator=torch.Generator(device="cpu").manual_seed(n)).to(DEV)
    acc = torch.empty(1, device=DEV)
    vals = set()
    for _ in range(5):
        K.sqnorm(x, acc)
        vals.add(acc.item())
    assert len(vals) == 1
    want = float(np.sum(x.cpu().numpy().astype(np.float64) ** 2))
    assert abs(vals.pop() - want) <= 1e-5 * want


def test_rag_mean_train_gradients():
    from src.autograd_ops import rag_mean_train
    from src.retrieval import PanelIndex
    rng = np.random.default_rng(4)
    D, L, n, n_ref, k, nq = 64, 1030, 300, 50, 4, 6
    panel = rng.integers(0, 2, (n_ref, n)).astype(np.uint8)
    pi = PanelIndex.from_alleles(panel, np.zeros(L, np.float32), DEV)
    idx = torch.from_numpy(rng.integers(0, n_ref, (nq, k))).to(DEV)
    W = torch.randn(12, D, device=DEV, requires_grad=True)
    Ar = torch.randn(L, D, device=DEV, requires_grad=True)
    pe = torch.randn(L, D, device=DEV)
    G = torch.randn(nq, L, D, device=DEV)
    out = rag_mean_train(W, Ar, idx, pi.codes, n, pe, L)
    (out.float() * G).sum().backward()
    toks = torch.zeros(n_ref, L, dtype=torch.long, device=DEV)
    toks[:, 0], toks[:, 1 + n] = 2, 3
    toks[:, 1:1 + n] = 5 + torch.from_numpy(panel).to(DEV).long()
    Wr = W.detach().clone().requires_grad_(True)
    Arr = Ar.detach().clone().requires_grad_(True)
    emb = torch.nn.functional.embedding(toks[idx], Wr, padding_idx=0)  # no gradient into <pad>
    ref = (emb + pe + Arr).mean(1)
    (ref * G.to(torch.bfloat16).float()).sum().backward()     # out is bf16: its incoming grad is too
    torch.testing.assert_close(out.float(), ref.detach(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(W.grad, Wr.grad, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(Ar.grad, Arr.grad, rtol=1e-5, atol=1e-4)


def _train_model(case):
    from src.model import build_model
    g = load_golden(case)
    cfg = g["cfg"]
    sd = golden_state_dict(cfg)
    m = build_model(cfg["vocab"], cfg["d"], cfg["layers"], cfg["heads"])
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m = m.to(DEV).train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    return g, cfg, m


def _train_inputs(g):
    x = {k: torch.from_numpy(np.ascontiguousarray(g[k])).to(DEV)
         for k in ("hap_1", "hap_2", "af", "af_p", "pos", "ref", "het", "hom", "mask",
                   "hap_1_label", "hap_2_label", "gt_label")}
    x["rag_emb_h1"] = torch.from_numpy(g["rag_mean_h1"]).to(DEV)[:, None]
    x["rag_emb_h2"] = torch.from_numpy(g["rag_mean_h2"]).to(DEV)[:, None]
    return x


def test_train_gradients_vs_reference_autograd():
    from src.autograd_ops import focal_loss
    g, cfg, m = _train_model("train_tiny")
    x = _train_inputs(g)
    out = m(x)
    mk = x["mask"].bool()
    l1 = focal_loss(out[0], x["hap_1_label"], mk, 2.0, 1.0)
    l2 = focal_loss(out[1], x["hap_2_label"], mk, 2.0, 1.0)
    lg = focal_loss(out[2], x["gt_label"], mk, 2.0, 1.0)
    total = 3 * l1 + 3 * l2 + 4 * lg
    total.backward()
    ref_losses = g["losses"]
    np.testing.assert_allclose([l1.item(), l2.item(), lg.item(), total.item()], ref_losses, rtol=1e-2)
    np.testing.assert_allclose(out[0].detach().cpu().numpy(), g["probs_h1"], atol=2e-2)
    np.testing.assert_allclose(out[2].detach().cpu().numpy(), g["gt"], atol=2e-2)
    named = dict(m.named_parameters())
    gnorm_all = math.sqrt(sum(float((g[k] ** 2).sum()) for k in g if k.startswith("g:")))
    checked, bad = 0, []
    for key in (k for k in g if k.startswith("g:")):
        name = key[2:]
        ref = torch.from_numpy(g[key]).to(DEV).double()
        p = named[name]
        got = p.grad.double() if p.grad is not None else torch.zeros_like(ref)
        rn = ref.norm().item()
        if rn < 1e-4 * gnorm_all:
            assert got.norm().item() <= 1e-3 * gnorm_all + 1e-6, name
            continue
        rel = ((got - ref).norm() / rn).item()
        cos = (got * ref).sum().item() / (got.norm().item() * rn + 1e-30)
        # the Fourier AF frequencies see the bf16 rounding of sin/cos(2 pi af f) amplified by 2 pi f
        lim, cmin = 8e-2, 0.99
        if name.endswith("basis_freqs"):
            lim = 0.15
        elif ".pos_feat." in name:
            # upstream of two batch-statistics BatchNorms (fusion.py:328-330): their backward
            # projects out the mean and x-hat components of the (bf16-noisy, ~2 %) incoming
            # gradient, so the small remainder carries a several-fold larger relative error
            lim, cmin = 0.5, 0.85
        print(f"{name:60s} rel {rel:.4f} cos {cos:.5f} |ref| {rn:.3e}")
        if not (rel <= lim and cos >= cmin):
            bad.append((name, rel, cos))
        checked += 1
    assert not bad, bad
    assert checked > 50
    # BatchNorm running statistics after the reference's four emb_fusion calls
    for key in (k for k in g if k.startswith("b:")):
        buf = dict(m.named_buffers())[key[2:]]
        np.testing.assert_allclose(buf.cpu().numpy(), g[key], rtol=1e-4, atol=1e-5)


def test_train_gradients_f32_mode_vs_reference_autograd():
    """The same train-mode graph in the f32 parity mode (autograd_ops.set_train_precision:
    exact-f32 MFMA Linear layers, f32 LayerNorm / attention): EVERY parameter gradient within
    1e-3 relative (Frobenius) of the reference's own autograd (train_tiny.npz), the losses within
    1e-5 and the outputs within 1e-5 — so a gradient bug of any size in any layer, BatchNorm
    path included, fails here rather than hiding in bf16 noise (the bf16 bar above stays)."""
    from src.autograd_ops import focal_loss, set_train_precision
    g, cfg, m = _train_model("train_tiny")
    x = _train_inputs(g)
    set_train_precision(torch.float32)
    try:
        out = m(x)
        mk = x["mask"].bool()
        l1 = focal_loss(out[0], x["hap_1_label"], mk, 2.0, 1.0)
        l2 = focal_loss(out[1], x["hap_2_label"], mk, 2.0, 1.0)
        lg = focal_loss(out[2], x["gt_label"], mk, 2.0, 1.0)
        total = 3 * l1 + 3 * l2 + 4 * lg
        total.backward()
    finally:
        set_train_precision(torch.bfloat16)
    np.testing.assert_allclose([l1.item(), l2.item(), lg.item(), total.item()], g["losses"], rtol=1e-5)
    np.testing.assert_allclose(out[0].detach().cpu().numpy(), g["probs_h1"], atol=1e-5)
    np.testing.assert_allclose(out[2].detach().cpu().numpy(), g["gt"], atol=1e-5)
    named = dict(m.named_parameters())
    gnorm_all = math.sqrt(sum(float((g[k] ** 2).sum()) for k in g if k.startswith("g:")))
    worst, checked = (0.0, None), 0
    for key in (k for k in g if k.startswith("g:")):
        name = key[2:]
        ref = torch.from_numpy(g[key]).to(DEV).double()
        p = named[name]
        got = p.grad.double() if p.grad is not None else torch.zeros_like(ref)
        rn = ref.norm().item()
        if rn < 1e-6 * gnorm_all:
            assert got.norm().item() <= 1e-5 * gnorm_all + 1e-9, name
            continue
        if name.endswith(("pos_feat.conv1.bias", "pos_feat.conv2.bias")):
            # a bias feeding a train-mode BatchNorm: the batch-mean subtraction cancels it, the
            # true gradient is 0 and both sides hold only rounding noise of the same size
            assert got.norm().item() <= 2 * rn + 1e-6 * gnorm_all, name
            continue
        rel = ((got - ref).norm() / rn).item()
        print(f"{name:60s} rel {rel:.2e} |ref| {rn:.3e}")
        worst = max(worst, (rel, name))
        checked += 1
    assert worst[0] <= 1e-3, worst
    assert checked > 50
    for key in (k for k in g if k.startswith("b:")):
        buf = dict(m.named_buffers())[key[2:]]
        np.testing.assert_allclose(buf.cpu().numpy(), g[key], rtol=1e-5, atol=1e-6)


def _v18_backward(precision):
    """The train_v18 fixture's loss through the train-mode graph in ``precision``; returns
    (fixture, model, outputs, losses)."""
    from src.autograd_ops import focal_loss, set_train_precision
    g, cfg, m = _train_model("train_v18")
    x = _train_inputs(g)
    set_train_precision(precision)
    try:
        out = m(x)
        mk = x["mask"].bool()
        ls = [focal_loss(out[0], x["hap_1_label"], mk, 2.0, 1.0), focal_loss(out[1], x["hap_2_label"], mk, 2.0, 1.0),
              focal_loss(out[2], x["gt_label"], mk, 2.0, 1.0)]
        total = 3 * ls[0] + 3 * ls[1] + 4 * ls[2]
        total.backward()
    finally:
        set_train_precision(torch.bfloat16)
    return g, m, out, [t.item() for t in ls] + [total.item()]


def _v18_layer_class(name: str) -> str:
    if ".transformer_blocks." in name:
        return "encoder." + ("attention" if ".attention." in name else "ffn" if ".feed_forward." in name else "norm")
    for key in ("emb_fusion", "rag_fusion", "hap_classifier", "gt_classifier", "embedding"):
        if key in name:
            return key
    return "other"


def test_train_v18_gradients_f32_mode_vs_reference_autograd():
    """configs[1]'s model (d384 / 12 layers / 12 heads, train_embedding_rag.py:41-43) in TRAIN mode
    (p = 0) on the exact-f32 parity path: every parameter gradient within 1e-3 relative of the
    reference's own autograd (tests/golden/train_v18.npz: norm, 16 seeded random projections and
    2048 sampled entries per parameter, tests/grad_sketch.py), losses within 1e-5, BatchNorm
    running statistics within 1e-5.  Reference: model/bert.py:148-219 under
    pretrain_with_val_optimized.py:212-235."""
    import grad_sketch as GS
    g, m, out, losses = _v18_backward(torch.float32)
    np.testing.assert_allclose(losses, g["losses"], rtol=1e-5)
    np.testing.assert_allclose(out[0].detach().cpu().numpy(), g["probs_h1"], atol=1e-5)
    np.testing.assert_allclose(out[2].detach().cpu().numpy(), g["gt"], atol=1e-5)
    named = dict(m.named_parameters())
    gnorm_all = math.sqrt(sum(float(g[f"gn:{n}"]) ** 2 for n in GS.names(g)))
    worst, checked = (0.0, None), 0
    for name in GS.names(g):
        p = named[name]
        got = p.grad.detach().float().cpu().numpy() if p.grad is not None else np.zeros(p.shape, np.float32)
        rn = float(g[f"gn:{name}"])
        if rn < 1e-6 * gnorm_all or name.endswith(("pos_feat.conv1.bias", "pos_feat.conv2.bias")):
            # no gradient, or a bias feeding a train-mode BatchNorm (true gradient 0, rounding noise)
            assert np.linalg.norm(got) <= 2 * rn + 1e-5 * gnorm_all, name
            continue
        est, rel_s, cos = GS.compare(name, got, g)
        worst = max(worst, (max(est, rel_s), name))
        checked += 1
    print("worst", worst, "checked", checked)
    assert worst[0] <= 1e-3, worst
    assert checked > 200
    for key in (k for k in g if k.startswith("b:")):
        buf = dict(m.named_buffers())[key[2:]]
        np.testing.assert_allclose(buf.cpu().numpy(), g[key], rtol=1e-5, atol=1e-6)


def test_train_v18_gradients_bf16_drift_bar():
    """The bf16 training graph the bench times (K = 384 stream GEMMs, the 128 x 128 dW splits,
    ln_bwd_pf at N = 1536, attn_bwd_*32) against the reference autograd at v18 size: per layer
    class, the gradient-norm-weighted relative error (estimated from the fixture's projections)
    stays under a drift bar; every parameter's sampled cosine >= 0.85 (the pos_feat BatchNorm
    stack excepted, see test_train_gradients_vs_reference_autograd).  The bar tracks bf16 drift
    as kernels change; exactness is the f32 test above."""
    import grad_sketch as GS
    g, m, out, losses = _v18_backward(torch.bfloat16)
    np.testing.assert_allclose(losses, g["losses"], rtol=3e-2)
    named = dict(m.named_parameters())
    num, den, bad = {}, {}, []
    for name in GS.names(g):
        p = named[name]
        rn = float(g[f"gn:{name}"])
        got = p.grad.detach().float().cpu().numpy() if p.grad is not None else np.zeros(p.shape, np.float32)
        if name.endswith("attention.linear_layers.1.bias"):
            # the key bias adds q . b_k to every score of a query: softmax cancels it, the true
            # gradient is 0 and both sides hold rounding noise (bf16 here: no direction to compare)
            wk = float(g[f"gn:{name[:-len('bias')]}weight"])
            print(f"{name}: |grad| {np.linalg.norm(got):.3e} (reference {rn:.3e}, key weight {wk:.3e})")
            assert np.linalg.norm(got) <= 0.05 * wk + 10 * rn, name
            continue
        est, rel_s, cos = GS.compare(name, got, g)
        c = _v18_layer_class(name)
        num[c] = num.get(c, 0.0) + (est * rn) ** 2
        den[c] = den.get(c, 0.0) + rn ** 2
        # (r4 box: the last layer's key weight 0.897, every other parameter >= 0.9)
        if ".pos_feat." not in name and rn > 0 and not name.endswith("basis_freqs") and cos < 0.85:
            bad.append((name, est, rel_s, cos))
    rel = {c: math.sqrt(num[c] / den[c]) for c in num if den[c] > 0}
    print({c: round(v, 4) for c, v in sorted(rel.items())})
    bars = {"encoder.attention": 0.08, "encoder.ffn": 0.08, "encoder.norm": 0.08, "emb_fusion": 0.15,
            "rag_fusion": 0.1, "hap_classifier": 0.08, "gt_classifier": 0.08, "embedding": 0.2, "other": 0.2}
    over = {c: v for c, v in rel.items() if v > bars[c]}
    assert not over and not bad, (over, bad)


def test_train_forward_matches_eval_engine_without_dropout():
    """Train-mode graph (p = 0, BatchNorm frozen) == the native eval forward (bf16)."""
    from src.engine import engine_for
    g, cfg, m = _train_model("train_tiny")
    x = _train_inputs(g)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm1d):
            mod.eval()
    with torch.no_grad():
        out_t = m(x)
        m.eval()
        eng = engine_for(m)
        eng.set_dtype(torch.bfloat16)
        out_e = m(x)
    for a, b in zip(out_t[:3], out_e[:3]):
        torch.testing.assert_close(a.float(), b.float(), rtol=3e-2, atol=3e-2)


def test_trainer_steps_reduce_loss_with_retrieval():
    """Synthetic dataset -> retrieval (train mode: indices + re-encode with grad) -> forward ->
    focal loss -> backward -> clip + fused Adam, repeated on one batch: the loss falls."""
    from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn
    from src.dataset.synthetic import make_rag_dataset
    from src.main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized
    from src.model import build_model
    torch.manual_seed(0)
    ds, vocab = make_rag_dataset(n_samples=4, n_sites=200, n_windows=1, n_ref_samples=32, seed=3, name="train")
    batch = embedding_rag_collate_fn([ds[i] for i in range(4)])
    m = build_model(len(vocab), 64, 2, 2).to(DEV)
    tr = BERTTrainerWithValidationOptimized(m, [batch], None, vocab, lr=2e-3, warmup_steps=1,
                                            grad_accum_steps=1, log_freq=0)
    tr.rag_train_dataset = ds
    tr.rag_k = 4
    losses = [tr.train_step(dict(batch)).item() for _ in range(12)]
    assert all(np.isfinite(losses))
    assert losses[-1] < 0.8 * losses[0], losses


@pytest.mark.parametrize("C", [2, 4])
def test_device_confusion_vs_oracle_cal_pr(C):
    """snvrag_confusion (DeviceConfusion) == cal_pr (optim_schedule.py:167-203) restated in the
    oracle, accumulated over two batches, with and without the rare/common second mask."""
    from src.main.optim_schedule import DeviceConfusion
    rng = np.random.default_rng(C)
    conf, conf2 = DeviceConfusion(C, DEV), DeviceConfusion(C, DEV)
    exp, exp2 = np.zeros((3, C), np.int64), np.zeros((3, C), np.int64)
    for b in range(2):
        probs = rng.random((3, 1030, C)).astype(np.float32)
        lab = rng.integers(0, C, (3, 1030))
        m = rng.random((3, 1030)) < 0.4
        m2 = rng.random((3, 1030)) < 0.5
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
        conf.update(T(probs), T(lab), T(m))
        conf2.update(T(probs), T(lab), T(m), T(m2 & m))
        exp += train_np.confusion(probs, lab, m, C)
        exp2 += train_np.confusion(probs, lab, m & m2, C)
    np.testing.assert_array_equal(conf.counts.cpu().numpy(), exp)
    np.testing.assert_array_equal(conf2.counts.cpu().numpy(), exp2)


def test_checkpoint_round_trip(tmp_path):
    """trainer.save -> a fresh trainer.load restores weights, the bf16 mirror, Adam moments and
    the LR-schedule step; the next training step then matches the uninterrupted run (up to the
    order of the loss kernel's float atomics)."""
    from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn
    from src.dataset.synthetic import make_rag_dataset
    from src.main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized
    from src.model import build_model
    ds, vocab = make_rag_dataset(n_samples=4, n_sites=200, n_windows=1, n_ref_samples=16, seed=3, name="train")
    batch = embedding_rag_collate_fn([ds[i] for i in range(4)])

    def trainer(seed):
        torch.manual_seed(seed)
        m = build_model(len(vocab), 64, 2, 2, dropout=0.0).to(DEV)
        t = BERTTrainerWithValidationOptimized(m, None, None, vocab, lr=1e-3, warmup_steps=5, log_freq=0)
        t.rag_train_dataset, t.rag_k = ds, 2
        return t
    a = trainer(0)
    for _ in range(2):
        a.train_step(dict(batch))
    path = a.save(1, str(tmp_path / "ck"))
    b = trainer(1)                                      # different init
    assert b.load(path) == 1
    for (ka, va), (kb, vb) in zip(a.model.state_dict().items(), b.model.state_dict().items()):
        assert ka == kb
        torch.testing.assert_close(va, vb, rtol=0, atol=0)
    assert b.optim_schedule.n_current_steps == a.optim_schedule.n_current_steps
    torch.manual_seed(123)                              # the GT head's FeedForward keeps dropout 0.1
    la = a.train_step(dict(batch))
    torch.manual_seed(123)
    lb = b.train_step(dict(batch))
    torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-5)
    for pa, pb in zip(a.model.parameters(), b.model.parameters()):
        torch.testing.assert_close(pb, pa, rtol=1e-4, atol=1e-6)


def test_neighbour_mean_dropout_semantics():
    """Per-neighbour dropout of the re-encoded neighbours (embedding_rag_dataset.py:404-417 +
    bert.py:171-183): p = 0 equals the counts/codes K-mean; p > 0 is unbiased (average over
    seeds -> the undropped mean) and differentiable in W and Ar."""
    from src.train_forward import neighbour_mean_dropout
    from src.autograd_ops import rag_mean_train
    rng = np.random.default_rng(0)
    nq, k, S, L, D = 6, 4, 200, 230, 32
    codes = torch.from_numpy((rng.random((50, 256)) < 0.3).astype(np.uint8)).to(DEV)
    idx = torch.from_numpy(rng.integers(0, 50, (nq, k))).to(DEV)
    idx[0, 3] = -1                                             # a missing neighbour
    W = torch.randn(12, D, device=DEV, requires_grad=True)
    Ar = torch.randn(L, D, device=DEV, requires_grad=True)
    pe = torch.randn(L, D, device=DEV)
    m0 = neighbour_mean_dropout(W, Ar, idx, codes, S, pe, L, 0.0).float()
    ref = rag_mean_train(W, Ar, idx, codes, S, pe, L).float()
    torch.testing.assert_close(m0, ref, rtol=2e-2, atol=2e-2)
    acc = torch.zeros_like(m0)
    torch.manual_seed(5)
    n = 200
    for _ in range(n):
        acc += neighbour_mean_dropout(W, Ar, idx, codes, S, pe, L, 0.3).float().detach()
    assert (acc / n - m0.detach()).abs().mean() < 0.05 * m0.abs().mean()
    out = neighbour_mean_dropout(W, Ar, idx, codes, S, pe, L, 0.3)
    out.float().sum().backward()
    assert W.grad[5].abs().sum() > 0 and W.grad[6].abs().sum() > 0 and W.grad[0].abs().sum() == 0
    assert Ar.grad.abs().sum() > 0


def test_train_mode_retrieval_query_dropout():
    """Train-mode retrieval embeds the queries with dropout (embedding_rag_dataset.py:385-386):
    with p = 0 the neighbours equal the eval search; with p = 0.1 they stay valid panel rows and
    mostly agree with the eval neighbours."""
    from src.dataset.synthetic import make_rag_dataset
    from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn
    from src.model import build_model
    ds, vocab = make_rag_dataset(n_samples=4, n_sites=300, n_windows=1, n_ref_samples=40, seed=2)
    torch.manual_seed(0)
    m = build_model(len(vocab), 64, 1, 4).to(DEV)
    batch = lambda: embedding_rag_collate_fn([ds[i] for i in range(4)])
    m.eval()
    ev = ds.process_batch_retrieval(batch(), m.bert.embedding, DEV, k_retrieve=4)["rag_idx_h1"]
    m.train()
    emb = m.bert.embedding
    emb.dropout.p = 0.0
    tr0 = ds.process_batch_retrieval(batch(), emb, DEV, k_retrieve=4)["rag_idx_h1"]
    torch.testing.assert_close(tr0, ev, rtol=0, atol=0)
    emb.dropout.p = 0.1
    tr = ds.process_batch_retrieval(batch(), emb, DEV, k_retrieve=4)["rag_idx_h1"]
    assert ((tr >= 0) & (tr < 80)).all()
    same = np.mean([len(set(a.tolist()) & set(b.tolist())) / 4 for a, b in zip(tr.cpu(), ev.cpu())])
    assert same >= 0.5


def test_train_mode_retrieval_lut_and_topk_bit_exact_vs_oracle(monkeypatch):
    """Train-mode retrieval ranks DROPPED-OUT query embeddings (embedding_rag_dataset.py:385-386:
    per-query offsets A_q != A_r, real-valued Delta) and, after a weight update inside the window,
    against the panel snapshot (Wp != W, :334-377).  Every LUT the device quantises equals the
    oracle's (Delta in the device's f32 arithmetic, oracle/lut_f32.c, then ``quantize_lut``) bit
    for bit, and the oracle's exact top-k from its OWN LUT equals the device's neighbours."""
    from oracle import knn_np
    from knn_helpers import decode_lut
    from src import kernels as Km
    from src.dataset.synthetic import make_rag_dataset
    from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn
    from src.model import build_model
    ds, vocab = make_rag_dataset(n_samples=6, n_sites=300, n_windows=1, n_ref_samples=50, seed=12, name="train")
    torch.manual_seed(3)
    m = build_model(len(vocab), 64, 1, 4).to(DEV).train()
    emb = m.bert.embedding
    emb.dropout.p = 0.1
    calls = []
    orig = Km.knn_lut

    def rec(tok_q, W, site_mask, n_sites, n_sites_pad, limbs=2, Aq=None, aq_period=0, Ar=None, tok0=5, tok1=6,
            mask_tok=4, Wp=None):
        out = orig(tok_q, W, site_mask, n_sites, n_sites_pad, limbs, Aq, aq_period, Ar, tok0, tok1, mask_tok, Wp=Wp)
        h = lambda t: None if t is None else t.detach().float().cpu().numpy()
        calls.append(dict(tok=tok_q.cpu().numpy(), W=h(W), Wp=h(Wp), Aq=h(Aq), aq_period=aq_period, Ar=h(Ar),
                          sm=site_mask.cpu().numpy()[:n_sites], limbs=limbs, pad=n_sites_pad,
                          lut=out[0].clone(), exps=out[1].cpu().numpy()))
        return out
    monkeypatch.setattr(Km, "knn_lut", rec)
    k, B = 5, 6
    batch = lambda: embedding_rag_collate_fn([ds[i] for i in range(B)])
    codes = ds.panel_index(0, DEV).codes.cpu().numpy()
    for step in range(2):
        calls.clear()
        b = ds.process_batch_retrieval(batch(), emb, DEV, k_retrieve=k)
        assert len(calls) == 1, len(calls)
        c = calls[0]
        assert c["Aq"] is not None                                   # the dropped-out query offsets
        if step == 1:
            assert c["Wp"] is not None and not np.array_equal(c["Wp"], c["W"])   # stale panel snapshot
        nq, S = c["tok"].shape[0], c["sm"].shape[0]
        delta = knn_np.lut_delta_f32(c["W"], c["tok"], c["sm"], Aq=c["Aq"], aq_period=c["aq_period"], Ar=c["Ar"],
                                     Wp=c["Wp"])
        dq_o, e_o = knn_np.quantize_lut(delta, c["limbs"])
        np.testing.assert_array_equal(c["exps"], e_o)
        np.testing.assert_array_equal(decode_lut(c["lut"], nq, c["pad"], c["limbs"])[:, :S], dq_o)
        oi, _ = knn_np.knn(codes[:, :S], dq_o, k)
        got = torch.cat([b["rag_idx_h1"], b["rag_idx_h2"]]).cpu().numpy()
        np.testing.assert_array_equal(got, oi)
        with torch.no_grad():                                        # a training step's update
            for p_ in emb.parameters():
                p_.add_(torch.randn_like(p_) * 0.2 * (p_.std() if p_.numel() > 1 else 1.0))


def test_train_panel_cache_window_snapshot_semantics():
    """panel_cache="window" (default): train-mode retrieval searches the panel embedded under the
    weights of the window's FIRST batch (the reference's JIT cache, embedding_rag_dataset.py:
    334-377, rebuilt only on a window change or a reset), while the queries are embedded under the
    current weights; "fresh" searches under the current weights.  Both checked against the
    reference algorithm written out in torch (eval-mode panel embedding, cdist, smallest k) after
    a weight update between two batches of one window; the overlap of the two neighbour sets is
    the staleness the reference trains with (printed)."""
    import copy
    from src.dataset.synthetic import make_rag_dataset
    from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn
    from src.model import build_model
    k, nb = 6, 4
    ds, vocab = make_rag_dataset(n_samples=nb, n_sites=300, n_windows=2, n_ref_samples=60, seed=5, name="train")
    torch.manual_seed(0)
    m = build_model(len(vocab), 64, 1, 4, dropout=0.0).to(DEV).train()
    emb = m.bert.embedding
    rows = [i for i in range(len(ds)) if ds[i]["window_idx"] == 0][:nb]
    batch = lambda: embedding_rag_collate_fn([ds[i] for i in rows])

    def reference_search(panel_emb_layer, query_emb_layer, b):
        """embedding_rag_dataset.py:339-402 in torch (float64 distances)."""
        toks = torch.as_tensor(ds.ref_tokens_complete[0], device=DEV)
        masked = ds._apply_mask_to_tokens_gpu(toks, torch.as_tensor(ds.window_masks[0], device=DEV))
        af_r = torch.as_tensor(ds.ref_af_windows[0], device=DEV).float().unsqueeze(0).expand(masked.shape[0], -1)
        was = [panel_emb_layer.training, query_emb_layer.training]
        panel_emb_layer.eval(); query_emb_layer.eval()
        with torch.no_grad():
            pe_ = panel_emb_layer(masked, af=af_r, pos=True).double().flatten(1)
            q = query_emb_layer(b["hap_1"].to(DEV), af=b["af"].to(DEV).float(), pos=True).double().flatten(1)
        panel_emb_layer.train(was[0]); query_emb_layer.train(was[1])
        d = torch.cdist(q, pe_)
        return d, d.topk(k, largest=False).values

    def check(idx, d, top):
        got = torch.gather(d, 1, idx).sort(1).values
        torch.testing.assert_close(got, top, rtol=1e-5, atol=1e-6)

    assert ds.panel_cache == "window"
    ds.clear_jit_cache()
    first = ds.process_batch_retrieval(batch(), emb, DEV, k_retrieve=k)        # snapshot taken here
    old = copy.deepcopy(emb)
    with torch.no_grad():                                                     # a training step's update
        for p_ in emb.parameters():
            p_.add_(torch.randn_like(p_) * 0.3 * (p_.std() if p_.numel() > 1 else 1.0))
    b = batch()
    stale = ds.process_batch_retrieval(b, emb, DEV, k_retrieve=k)["rag_idx_h1"]
    d_stale, top_stale = reference_search(old, emb, b)
    check(stale, d_stale, top_stale)
    ds.panel_cache = "fresh"
    fresh = ds.process_batch_retrieval(batch(), emb, DEV, k_retrieve=k)["rag_idx_h1"]
    d_fresh, top_fresh = reference_search(emb, emb, b)
    check(fresh, d_fresh, top_fresh)
    overlap = np.mean([len(set(a.tolist()) & set(c.tolist())) / k for a, c in zip(stale.cpu(), fresh.cpu())])
    print(f"neighbour overlap, snapshot vs current panel embedding after one update: {overlap:.3f}")
    # a window change rebuilds the snapshot (jit_cache_win_idx != win_idx): back on window 0 the
    # panel side is the current weights again
    ds.panel_cache = "window"
    other = [i for i in range(len(ds)) if ds[i]["window_idx"] == 1][:2]
    ds.process_batch_retrieval(embedding_rag_collate_fn([ds[i] for i in other]), emb, DEV, k_retrieve=k)
    again = ds.process_batch_retrieval(batch(), emb, DEV, k_retrieve=k)["rag_idx_h1"]
    check(again, d_fresh, top_fresh)
    assert first["rag_idx_h1"].shape == (nb, k)


def _ref_trainer_handoff(data, device):
    """pretrain_with_val_optimized.py:180-195 — the reference trainer copies these keys to the
    device and forwards ONLY rag_emb_h1/h2 of what retrieval added."""
    gpu = {k: data[k].to(device, dtype=torch.long if k.startswith("hap") else torch.float)
           for k in ("hap_1", "hap_2", "pos", "af", "af_p", "ref", "het", "hom")}
    if "rag_emb_h1" in data:
        gpu["rag_emb_h1"] = data["rag_emb_h1"]
    if "rag_emb_h2" in data:
        gpu["rag_emb_h2"] = data["rag_emb_h2"]
    return gpu


def test_train_retrieval_contract_through_reference_handoff():
    """Train-mode process_batch_retrieval adds autograd-connected f32 rag_emb_h1/h2 [B, 1, L, D]
    (embedding_rag_dataset.py:404-442), so a batch handed over the reference trainer's way
    (:172-195) trains WITH the neighbours: the loss differs from the no-RAG forward and the
    token table's gradient carries the neighbour path's contribution (= the total minus the
    gradient with rag_emb detached, which must be non-zero on the allele rows)."""
    from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn
    from src.dataset.synthetic import make_rag_dataset
    from src.autograd_ops import focal_loss
    from src.model import build_model
    torch.manual_seed(0)
    ds, vocab = make_rag_dataset(n_samples=4, n_sites=200, n_windows=1, n_ref_samples=24, seed=3, name="train")
    m = build_model(len(vocab), 64, 2, 2, dropout=0.0).to(DEV).train()
    emb = m.bert.embedding
    W = emb.tokenizer.weight
    batch = embedding_rag_collate_fn([ds[i] for i in range(4)])
    with torch.enable_grad():                                          # :170-177
        data = ds.process_batch_retrieval(batch, emb, DEV, k_retrieve=4)
    r1 = data["rag_emb_h1"]
    assert r1.shape == (4, 1, 1030, 64) and r1.dtype == torch.float32 and r1.requires_grad
    gpu = _ref_trainer_handoff(data, DEV)
    mk = data["mask"].to(DEV).bool()

    def loss_of(x):
        out = m(x)
        return (3 * focal_loss(out[0], data["hap_1_label"].to(DEV), mk) + 3 * focal_loss(out[1], data["hap_2_label"].to(DEV), mk)
                + 4 * focal_loss(out[2], data["gt_label"].to(DEV), mk))
    loss = loss_of(gpu)
    g_total, G1, G2 = torch.autograd.grad(loss, [W, gpu["rag_emb_h1"], gpu["rag_emb_h2"]])
    det = dict(gpu, rag_emb_h1=gpu["rag_emb_h1"].detach(), rag_emb_h2=gpu["rag_emb_h2"].detach())
    (g_query,) = torch.autograd.grad(loss_of(det), W)
    norag = {k: v for k, v in gpu.items() if not k.startswith("rag")}
    loss0 = loss_of(norag)
    assert abs(loss.item() - loss0.item()) > 1e-4 * abs(loss0.item()), (loss.item(), loss0.item())
    g_nb = g_total - g_query
    assert g_nb[5].abs().sum() > 0 and g_nb[6].abs().sum() > 0        # allele rows via the neighbours
    assert g_nb[0].abs().sum() == 0                                    # <pad>: padding_idx
    # the neighbour gradient equals autograd through the reference's own K-mean formula
    idx = torch.cat([data["rag_idx_h1"], data["rag_idx_h2"]])
    codes = ds.panel_index(0, DEV).codes
    tok = torch.zeros(*idx.shape, 1030, dtype=torch.long, device=DEV)
    tok[..., 0], tok[..., 201] = 2, 3
    tok[..., 1:201] = 5 + codes[idx][..., :200].long()
    Wr = W.detach().clone().requires_grad_(True)
    with torch.no_grad():
        from src.train_forward import af_embedding
        Ar = af_embedding(emb.af_embedding, torch.from_numpy(ds.ref_af_windows[0]).to(DEV).view(1, -1))[0].float()
    ref = (torch.nn.functional.embedding(tok, Wr, padding_idx=0) + emb.position.pe[0, :1030] + Ar).mean(1)
    torch.testing.assert_close(torch.cat([r1[:, 0], data["rag_emb_h2"][:, 0]]).detach(), ref.detach(),
                               rtol=2e-2, atol=2e-2)
    (g_ref,) = torch.autograd.grad((ref * torch.cat([G1, G2])[:, 0]).sum(), Wr)
    torch.testing.assert_close(g_nb[[2, 3, 5, 6]], g_ref[[2, 3, 5, 6]], rtol=5e-2,
                               atol=2e-2 * g_ref.abs().max().item())


def test_train_retrieval_dense_and_shared_neighbour_dropout():
    """dense=True in train mode returns the reference's [B, k, L, D] per-neighbour embeddings
    whose mean over k is the K-mean; with dropout every retrieved haplotype of a window is
    re-encoded ONCE (embedding_rag_dataset.py:406-417), so two queries that retrieved the same
    haplotype see the identical dropped-out embedding, and the dropout is unbiased."""
    from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn
    from src.dataset.synthetic import make_rag_dataset
    from src.model import build_model
    torch.manual_seed(1)
    ds, vocab = make_rag_dataset(n_samples=6, n_sites=150, n_windows=1, n_ref_samples=6, seed=4, name="train")
    m = build_model(len(vocab), 64, 1, 2, dropout=0.0).to(DEV).train()
    emb = m.bert.embedding
    batch = lambda: embedding_rag_collate_fn([ds[i] for i in range(6)])
    d0 = ds.process_batch_retrieval(batch(), emb, DEV, k_retrieve=4, dense=True)
    k0 = ds.process_batch_retrieval(batch(), emb, DEV, k_retrieve=4)
    assert d0["rag_emb_h1"].shape == (6, 4, 1030, 64)
    torch.testing.assert_close(d0["rag_emb_h1"].mean(1), k0["rag_emb_h1"][:, 0], rtol=2e-2, atol=2e-2)
    emb.dropout.p = 0.3
    d = ds.process_batch_retrieval(batch(), emb, DEV, k_retrieve=4, dense=True)
    e = torch.cat([d["rag_emb_h1"], d["rag_emb_h2"]]).detach()
    idx = torch.cat([d["rag_idx_h1"], d["rag_idx_h2"]])
    flat_i, flat_e = idx.reshape(-1), e.reshape(-1, 1030, 64)
    pairs = 0
    for a in range(flat_i.numel()):
        for b in range(a + 1, flat_i.numel()):
            if flat_i[a] == flat_i[b] and a // 4 != b // 4:
                assert torch.equal(flat_e[a], flat_e[b])
                pairs += 1
    assert pairs > 0                                      # 12 panel haplotypes, 48 picks: repeats
    zero = (e == 0).float().mean().item()
    assert 0.2 < zero < 0.4                               # ~p of the entries dropped


def test_train_entry_point_save_best_and_resume(tmp_path, capsys):
    """src/train_embedding_rag.main end to end (train_embedding_rag.py:343-434): two epochs of
    retrieval + training + validation on synthetic data, per-epoch checkpoints, .best.pth, the
    reference's CSV columns (train and val rows per epoch), then a resume from epoch 0's
    checkpoint that restores the curriculum level, optimizer / schedule / sampler state and
    continues at epoch 1."""
    import csv
    from src import train_embedding_rag as T
    out = tmp_path / "rag_bert.model"
    mcsv = tmp_path / "metrics.csv"
    common = ["--synthetic", "4", "--synthetic_sites", "120", "--synthetic_windows", "2", "--synthetic_ref", "12",
              "--dims", "64", "--layers", "1", "--attn_heads", "2", "--train_batch_size", "2",
              "--val_batch_size", "2", "--max_steps", "2", "--log_freq", "1", "--warmup_steps", "3",
              "--rag_k", "3", "--output_path", str(out), "--metrics_csv", str(mcsv)]
    tr = T.main(common + ["--epochs", "2"])
    for suffix in (".ep0", ".ep1", ".best.pth"):
        assert (tmp_path / f"rag_bert.model{suffix}").exists(), suffix
    with open(mcsv) as f:
        rows = list(csv.DictReader(f))
    assert list(rows[0]) == ["epoch", "mode", "loss", "accuracy", "overall_f1", "overall_precision",
                             "overall_recall", "rare_f1", "rare_precision", "rare_recall", "common_f1",
                             "common_precision", "common_recall"]
    assert [(r["epoch"], r["mode"]) for r in rows] == [("1", "train"), ("1", "val"), ("2", "train"), ("2", "val")]
    assert all(0.0 <= float(r["overall_f1"]) <= 1.0 for r in rows)
    steps = tr.optim_schedule.n_current_steps
    assert steps >= 2
    assert tr.train_data.dataset._level == 1                  # add_level after epoch 1 ((1 + 1) % 2 == 0)
    ck = torch.load(str(out) + ".ep0", map_location="cpu", weights_only=True)
    assert {"model", "optim", "schedule_steps", "epoch", "sampler"} <= set(ck)
    tr2 = T.main(common + ["--epochs", "2", "--resume_path", str(out) + ".ep0"])
    assert tr2.optim_schedule.n_current_steps > ck["schedule_steps"]
    assert tr2.train_data.dataset._level == 1                 # min(1 // 2, 7) restored, +1 after epoch 1
    with open(mcsv) as f:
        rows2 = list(csv.DictReader(f))
    assert [(r["epoch"], r["mode"]) for r in rows2[4:]] == [("2", "train"), ("2", "val")]


def test_train_entry_point_resume_from_reference_checkpoint(tmp_path):
    """Resume from the reference trainer's own checkpoint object (a pickled BERTFoundationModel,
    tests/golden/ref_module_tiny.pth) and from a plain state_dict: the weights load, and the run
    starts at --resume_epoch as the reference does (train_embedding_rag.py:155-191, default 0) —
    an explicit 0 included, and not after an epoch the file does not hold; a checkpoint of this
    trainer without --resume_epoch continues after its saved epoch."""
    import csv
    import os
    from src import train_embedding_rag as T
    from src.model.checkpoint import load_state_dict_any
    pth = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_module_tiny.pth")
    torch.save({"state_dict": load_state_dict_any(pth), "epoch": 5}, tmp_path / "sd_epoch5.pt")
    out = tmp_path / "m.model"
    mcsv = tmp_path / "metrics.csv"
    common = ["--synthetic", "4", "--synthetic_sites", "120", "--synthetic_windows", "1", "--synthetic_ref", "12",
              "--dims", "64", "--layers", "2", "--attn_heads", "2", "--train_batch_size", "2",
              "--val_batch_size", "2", "--max_steps", "1", "--log_freq", "1", "--warmup_steps", "3",
              "--rag_k", "3", "--output_path", str(out), "--metrics_csv", str(mcsv), "--epochs", "1"]

    def epochs_run():
        with open(mcsv) as f:
            rows = list(csv.DictReader(f))
        os.remove(mcsv)
        return sorted({int(r["epoch"]) for r in rows})
    for path, extra in ((pth, []), (pth, ["--resume_epoch", "0"]), (str(tmp_path / "sd_epoch5.pt"), [])):
        tr = T.main(common + ["--resume_path", path] + extra)
        assert tr.loaded_own_checkpoint is False
        assert epochs_run() == [1]                               # epoch 0 ran (CSV epochs are 1-based)
    # the run above saved <out>.ep0, a checkpoint of this trainer: unset --resume_epoch continues after it
    tr = T.main(common[:-1] + ["2", "--resume_path", str(out) + ".ep0"])
    assert tr.loaded_own_checkpoint is True
    assert epochs_run() == [2]
    tr = T.main(common[:-1] + ["2", "--resume_path", str(out) + ".ep0", "--resume_epoch", "0"])
    assert epochs_run() == [1, 2]


def test_direct_weight_grads_match_autograd_accumulation():
    """autograd_ops.direct_weight_grads (the trainer's backward): Linear dW / db accumulated by
    the dW kernel straight into the FlatParams gradient buffer equal autograd's own
    accumulation of the returned gradients, including a second micro-batch on top of the first
    (gradient accumulation); every parameter's post-accumulate hook (GradBucketer's readiness
    signal) fires exactly once per backward on both paths."""
    from src import autograd_ops as A
    from src.main.optimizer import FlatParams
    from src.model import build_model
    g = load_golden("train_tiny")
    torch.manual_seed(3)
    m = build_model(g["cfg"]["vocab"], 128, 1, 2, dropout=0.0).to(DEV).train()   # D % 128 == 0
    x = _train_inputs(g)
    B, L = x["hap_1"].shape
    for k in ("rag_emb_h1", "rag_emb_h2"):
        x[k] = torch.randn(B, 1, L, 128, device=DEV) * 0.5
    fp = FlatParams(m.parameters())
    reports = {}                        # post-accumulate hook calls per parameter (GradBucketer's signal)
    hooks = [p.register_post_accumulate_grad_hook(lambda _p, k=i: reports.__setitem__(k, reports.get(k, 0) + 1))
             for i, p in enumerate(fp.params)]

    def once():                         # every parameter in the graph reported exactly once
        ok = len(reports) > 50 and set(reports.values()) == {1}
        reports.clear()
        return ok

    def loss():
        from src.autograd_ops import focal_loss
        out = m(x)
        mk = x["mask"].bool()
        return 3 * focal_loss(out[0], x["hap_1_label"], mk, 2.0, 1.0) + 4 * focal_loss(out[2], x["gt_label"], mk, 2.0, 1.0)

    fp.zero_grad()
    loss().backward()
    ref = fp.grad.clone()
    assert once()
    fp.zero_grad()
    loss().backward()
    floor = ((fp.grad - ref).norm() / ref.norm()).item()   # run-to-run (float atomics)
    assert once()
    fp.zero_grad()
    with A.direct_weight_grads():
        loss().backward()
    got = fp.grad.clone()
    assert once()
    names = {id(p): n for n, p in m.named_parameters()}
    worst = sorted(((((fp.view(got, i) - fp.view(ref, i)).norm() / (fp.view(ref, i).norm() + 1e-30)).item(),
                     names[id(p)]) for i, p in enumerate(fp.params)), reverse=True)[:8]
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 1e-5 + 10 * floor, (rel, floor, worst)
    with A.direct_weight_grads():
        loss().backward()
    rel2 = ((fp.grad - 2 * ref).norm() / (2 * ref).norm()).item()
    worst2 = sorted(((((fp.view(fp.grad, i) - 2 * fp.view(ref, i)).norm() / (2 * fp.view(ref, i).norm() + 1e-30)).item(),
                      names[id(p)]) for i, p in enumerate(fp.params)), reverse=True)[:8]
    assert rel2 < 1e-5 + 10 * floor, (rel2, floor, worst2)
    assert once()
    for h in hooks:
        h.remove()


def test_stream_gemm_repacks_after_optimizer_step():
    """The K = 384 stream-GEMM weight packs (autograd_ops._sg_stream / _sg_stream_t: forward and
    dX) are cached per parameter version and optimizer epoch: after a FusedAdam step on the flat
    buffer (a HIP kernel, outside torch's version counter) the next forward and backward use the
    updated weights, not the stale packs."""
    from src.autograd_ops import hip_linear
    from src.main.optimizer import FlatParams, FusedAdam
    torch.manual_seed(7)
    lin = torch.nn.Linear(384, 384).to(DEV)
    fp = FlatParams(lin.parameters())
    opt = FusedAdam(fp, lr=0.05)
    x = torch.randn(2048, 384, device=DEV).to(torch.bfloat16).requires_grad_(True)

    def check():
        x.grad = None
        y = hip_linear(x, lin.weight, lin.bias)
        w = lin.weight.detach().to(torch.bfloat16).float()
        ref = x.detach().float() @ w.t() + lin.bias.detach()
        assert ((y.float() - ref).norm() / ref.norm()).item() < 1e-2
        g = torch.randn_like(y)
        y.backward(g)
        gx_ref = g.float() @ w
        assert ((x.grad.float() - gx_ref).norm() / gx_ref.norm()).item() < 1e-2

    check()
    before = lin.weight.detach().clone()
    fp.grad.normal_()
    opt.step()
    assert (lin.weight.detach() - before).abs().max().item() > 1e-3     # the weights moved
    check()


def test_derived_weights_refresh_in_one_launch():
    """Stream-GEMM packs, transposed / concatenated bf16 copies and bias tables of f32 master
    weights (autograd_ops' derived registry, csrc/sgemm.hip derive_kernel) equal the torch
    formulas they replace — at creation, after an optimizer-style raw update + weights_updated()
    (one refresh launch for all), and after a torch in-place update (refreshed at next use)."""
    from src import autograd_ops as A
    from src import kernels as K
    g = torch.Generator(device="cpu").manual_seed(11)
    q, k, v = (torch.nn.Parameter(torch.randn(384, 384, generator=g).to(DEV)) for _ in range(3))
    bq, bk, bv = (torch.nn.Parameter(torch.randn(384, generator=g).to(DEV)) for _ in range(3))
    W = torch.nn.Parameter(torch.randn(1536, 386, generator=g).to(DEV))     # rank-2 layer [W | c1 c2]
    b = torch.nn.Parameter(torch.randn(1536, generator=g).to(DEV))
    A.clear_weight_cache()

    def check():
        bf = lambda t: t.detach().to(torch.bfloat16)
        pk, vec = A._sg_stream([q, k, v], [bq, bk, bv], 1152)
        assert torch.equal(pk, K.sgemm_pack(torch.cat([bf(q), bf(k), bf(v)])))
        assert torch.equal(vec, torch.cat([bq, bk, bv]).detach())
        pk2, vec2 = A._sg_stream([W[:, :384]], [b], 1536, extra=(W[:, 384], W[:, 385]))
        assert torch.equal(pk2, K.sgemm_pack(bf(W[:, :384]).contiguous()))
        assert torch.equal(vec2, torch.cat([b, W[:, 384], W[:, 385]]).detach())
        pt, z = A._sg_stream_t(q, 384)
        assert torch.equal(pt, K.sgemm_pack(bf(q).t().contiguous())) and not z.any()
        assert torch.equal(A._cat_bf16([q, k, v]), torch.cat([bf(q), bf(k), bf(v)]))
        assert torch.equal(A._cat_bf16([q, k, v], transposed=True), torch.cat([bf(q), bf(k), bf(v)]).t())
        assert torch.equal(A._cat_f32([bq, bk, bv]), torch.cat([bq, bk, bv]).detach())
        assert torch.equal(A.bf16_of(W[:, :384]), bf(W[:, :384]))
        assert torch.equal(A.bf16_of(q, transposed=True), bf(q).t())

    check()
    n0 = len(A._DER)
    for t in (q, k, v, bq, bk, bv, W, b):          # a raw update (no version bump), like FusedAdam
        t.data.add_(0.25)
    A.weights_updated()
    assert len(A._DER) == n0
    check()
    with torch.no_grad():                            # a torch update: version bump, refreshed at use
        k.mul_(-1.5)
        W.add_(1.0)
    check()
    A.clear_weight_cache()


@pytest.mark.parametrize("N", [128, 384, 512])
def test_ln_forward_row_groups_match_one_row_per_wave(N):
    """The 16-lane row-group LayerNorm forward (N <= 512) against the one-row-per-wave kernel on
    the same inputs, with residual dropout + activation and output dropout: same masks, outputs
    within one bf16 rounding, statistics to f32 summation order; M not a multiple of 16."""
    from src import kernels as K
    M = 1000 * 4 + 13
    g = torch.Generator(device="cpu").manual_seed(N)
    x, r = (torch.randn(M, N, generator=g).to(DEV).bfloat16() for _ in range(2))
    w, b = torch.randn(N, generator=g).to(DEV), torch.randn(N, generator=g).to(DEV)
    outs = []
    for rows1 in (0, 1):
        with K.option("ln_rows1", rows1):
            outs.append(K.ln_fwd_train(x, r, w, b, 1e-5, p_r=0.1, p_out=0.19, seed=9, slope_r=0.1))
    (y0, s0, st0), (y1, s1, st1) = outs
    assert torch.equal(s0, s1)
    torch.testing.assert_close(st0, st1, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(y0.float(), y1.float(), rtol=1e-2, atol=1e-2)
    assert ((y0 == 0) == (y1 == 0)).all()                    # the same dropped elements


@pytest.mark.parametrize("M,Kd", [(0, 1536), (1, 1536), (777, 1536), (49440 // 8 + 5, 1536), (3001, 1024),
                                  (5, 40)])
def test_head2_linear_vs_torch_fp32(M, Kd):
    """The hap head's Linear(4D, 2) kernels (forward, dx, dW with direct .grad accumulation)
    against torch fp32 on the same bf16 activations: logits / dW / db to f32 summation order
    (tolerance 1e-4 relative), dx within one bf16 rounding.  K = 1536 (the model's 4D) runs the
    wave-per-16-rows forward, other K the generic one."""
    from src import autograd_ops as A
    g = torch.Generator(device="cpu").manual_seed(M)
    lin = torch.nn.Linear(Kd, 2).to(DEV)
    x = torch.randn(M, Kd, generator=g).to(DEV).bfloat16().requires_grad_(True)
    gy = torch.randn(M, 2, generator=g).to(DEV)
    y = A.head2_linear(x, lin)
    assert y.dtype == torch.float32 and y.shape == (M, 2)
    xr = x.detach().float().requires_grad_(True)
    w = lin.weight.detach().clone().requires_grad_(True)
    b = lin.bias.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.linear(xr, w, b)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    y.backward(gy)
    yr.backward(gy)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(lin.weight.grad, w.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(lin.bias.grad, b.grad, rtol=1e-4, atol=1e-3)
    # direct accumulation into existing .grad buffers (the trainer's flat gradient buffer)
    gw0, gb0 = lin.weight.grad.clone(), lin.bias.grad.clone()
    with A.direct_weight_grads():
        A.head2_linear(x.detach(), lin).backward(gy)
    torch.testing.assert_close(lin.weight.grad, gw0 + w.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(lin.bias.grad, gb0 + b.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("M,V,D,pad", [(0, 10, 384, 0), (1, 10, 384, 0), (49440 // 4 + 3, 10, 384, 0),
                                       (777, 16, 6, None), (300, 1, 2, None)])
def test_token_table_gradient_vs_onehot_fp64(M, V, D, pad):
    """The token-table weight gradient kernel (tiny_embedding's backward) against the one-hot
    product in float64: the padding row gets nothing, float32 summation-order tolerance, and two
    calls on the same inputs agree bitwise (fixed-order reduction)."""
    from src import autograd_ops as A, kernels as K
    g = torch.Generator(device="cpu").manual_seed(M + V)
    tok = torch.randint(0, V, (M,), generator=g)
    gy = torch.randn(M, D, generator=g)
    want = torch.nn.functional.one_hot(tok, V).double().t() @ gy.double()
    if pad is not None:
        want[pad] = 0
    got = K.tokgrad(tok.to(DEV), gy.to(DEV), V, pad)
    torch.testing.assert_close(got.cpu().double(), want, rtol=1e-5, atol=1e-4)
    assert torch.equal(got, K.tokgrad(tok.to(DEV), gy.to(DEV), V, pad))
    if M:                                   # through the autograd node
        W = torch.randn(V, D, device=DEV, requires_grad=True)
        A.tiny_embedding(tok.to(DEV), W, pad).backward(gy.to(DEV))
        torch.testing.assert_close(W.grad.cpu().double(), want, rtol=1e-5, atol=1e-4)


def _configs1_case():
    """configs[1] at its real shape (train_embedding_rag.py defaults; the bench's training leg):
    B = 24 samples, a 512-site window (L = 1030 tokens), k = 8 neighbours from a 10 000-haplotype
    panel, d384 / 12 layers / 12 heads, TRAIN mode with every dropout at p = 0.  Retrieval runs
    once (the trainer's own process_batch_retrieval); its neighbour means are then held fixed, so
    the loss is a smooth function of the weights for the finite differences below."""
    from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn
    from src.dataset.synthetic import make_rag_dataset
    from src.model import build_model
    # (the epoch-0 window masks come from numpy's global RNG, as in the reference — the CLI seeds it
    # first, train_embedding_rag.py main; unseeded, two processes retrieve different neighbours)
    st = np.random.get_state()
    np.random.seed(0)
    ds, vocab = make_rag_dataset(n_samples=24, n_sites=512, n_windows=1, n_ref_samples=5000, seed=7, name="train")
    np.random.set_state(st)
    batch = embedding_rag_collate_fn([ds[i] for i in range(24)])
    torch.manual_seed(0)
    m = build_model(len(vocab), 384, 12, 12).to(DEV).train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    data = ds.process_batch_retrieval(dict(batch), m.bert.embedding, DEV, k_retrieve=8)
    x = {k: (v.to(DEV) if torch.is_tensor(v) else v) for k, v in data.items()}
    x["rag_emb_h1"], x["rag_emb_h2"] = x["rag_emb_h1"].detach(), x["rag_emb_h2"].detach()
    return m, x


def _configs1_loss(m, x):
    from src.autograd_ops import focal_loss
    out = m(x)
    mk = x["mask"].bool()
    return (3 * focal_loss(out[0], x["hap_1_label"], mk, 2.0, 1.0) + 3 * focal_loss(out[1], x["hap_2_label"], mk, 2.0, 1.0)
            + 4 * focal_loss(out[2], x["gt_label"], mk, 2.0, 1.0))


def test_train_configs1_shape_directional_derivatives_and_bf16_drift():
    """configs[1] at full size (the shape the bench's training leg times), checked without a
    reference run (the reference's autograd at B = 24, L = 1030 needs ~60 GB of host memory for
    its attention matrices; the fixture-size tests pin it against the reference itself):
      * exact-f32 mode: the gradient's directional derivative along its own direction, overall and
        restricted to each layer class, equals the central finite difference of the loss
        to 1.5e-3 (a wrong gradient — direction or scale — moves the difference quotient off |g|);
      * the bf16 product path: loss within 1e-3 of f32, every layer class's gradient within a
        relative error of 0.05 and cosine >= 0.999 of the f32 gradient (measured r6: 1e-4; rel
        0.8e-3 - 1.3e-2, cos >= 0.99992)."""
    from src import autograd_ops as AO
    m, x = _configs1_case()
    params = [(n, p) for n, p in m.named_parameters() if p.requires_grad]
    AO.set_train_precision(torch.float32)
    try:
        m.zero_grad(set_to_none=True)
        L0 = _configs1_loss(m, x)
        L0.backward()
        g32 = {n: (p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p)) for n, p in params}

        def loss_at(step, d):
            with torch.no_grad():
                for n, p in params:
                    if n in d:
                        p.add_(d[n], alpha=step)
            AO.weights_updated()
            with torch.no_grad():
                v = float(_configs1_loss(m, x))
            with torch.no_grad():
                for n, p in params:
                    if n in d:
                        p.add_(d[n], alpha=-step)
            AO.weights_updated()
            return v

        groups = {"all": [n for n, _ in params]}
        for n, _ in params:
            groups.setdefault(_v18_layer_class(n), []).append(n)
        L0v = float(L0.detach())
        for gname, names in groups.items():
            gn = math.sqrt(sum(float((g32[n].double() ** 2).sum()) for n in names))
            if gn < 1e-6 * abs(L0v):
                continue
            d = {n: (g32[n] / gn) for n in names}
            # step: a loss change of 2e-3 relative each way.  Measured (r6, profiles/r6_train_configs1_fd.txt):
            # the difference quotient converges to |g| as the step shrinks (rel +1.5e-3 / +5e-4 / +2e-4
            # at 8e-3 / 2e-3 / 5e-4: the curvature term), the loss repeats to 2e-7, so the noise floor
            # of the quotient is ~4e-4 at 5e-4
            eps = 2e-3 * abs(L0v) / gn
            fd = (loss_at(eps, d) - loss_at(-eps, d)) / (2 * eps)
            print(f"{gname:18s} |g| {gn:.6e}  finite difference {fd:.6e}  rel {(fd - gn) / gn:+.2e}")
            assert abs(fd - gn) <= 1.5e-3 * gn, (gname, fd, gn)
    finally:
        AO.set_train_precision(torch.bfloat16)
    m.zero_grad(set_to_none=True)
    AO.weights_updated()
    L16 = _configs1_loss(m, x)
    L16.backward()
    print(f"loss f32 {L0v:.4f} bf16 {float(L16.detach()):.4f}")
    assert abs(float(L16.detach()) - L0v) <= 1e-3 * abs(L0v)
    num, den, dot, n16 = {}, {}, {}, {}
    for n, p in params:
        c = _v18_layer_class(n)
        a = g32[n].double()
        b = p.grad.detach().double() if p.grad is not None else torch.zeros_like(a)
        num[c] = num.get(c, 0.0) + float(((b - a) ** 2).sum())
        den[c] = den.get(c, 0.0) + float((a ** 2).sum())
        dot[c] = dot.get(c, 0.0) + float((a * b).sum())
        n16[c] = n16.get(c, 0.0) + float((b ** 2).sum())
    for c in sorted(num):
        rel = math.sqrt(num[c] / max(den[c], 1e-30))
        cos = dot[c] / math.sqrt(max(den[c] * n16[c], 1e-30))
        print(f"bf16 vs f32 {c:18s} rel {rel:.3e} cos {cos:.6f}")
        assert rel <= 0.05 and cos >= 0.999, (c, rel, cos)
