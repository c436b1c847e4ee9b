"""Host restatement of the attention-dropout keep mask (csrc/attn_common.h) for the parity tests:
h(q, j) = mix24(base + q * 0x9E3779B1 + j * 0x85EBCA77), base = fmix32(lo(seed) ^ fmix32(hi(seed) +
sh * 0xC2B2AE3D)); key k uses 16-bit half (k & 1) of h(q, k >> 1); keep iff that half >=
round(p * 2^16) (at least 1 when p > 0).  mix24 = lowbias32 with 24-bit multiplies."""
import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def fmix32(h):
    h = np.asarray(h, np.uint64) & M32
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & M32
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & M32
    h ^= h >> np.uint64(16)
    return h


def mix24(h):
    h = np.asarray(h, np.uint64) & M32
    h ^= h >> np.uint64(16)
    h = ((h & np.uint64(0xFFFFFF)) * np.uint64(0xEB352D)) & M32
    h ^= h >> np.uint64(15)
    h = ((h & np.uint64(0xFFFFFF)) * np.uint64(0x6CA68B)) & M32
    h ^= h >> np.uint64(16)
    return h


def keep_mask(seed: int, nseq: int, heads: int, L: int, p: float) -> np.ndarray:
    """bool [nseq, heads, L(q), L(k)]"""
    thresh = np.uint64(max(1, int(p * 65536.0 + 0.5))) if p > 0 else np.uint64(0)
    lo, hi = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    q = np.arange(L, dtype=np.uint64)
    out = np.zeros((nseq, heads, L, L), bool)
    for sq in range(nseq):
        for h in range(heads):
            sh = np.uint64(sq * heads + h)
            base = fmix32(lo ^ fmix32((hi + sh * np.uint64(0xC2B2AE3D)) & M32))
            x = (base + q[:, None] * np.uint64(0x9E3779B1) + (q[None, :] >> np.uint64(1)) * np.uint64(0x85EBCA77)) & M32
            hh = mix24(x)
            half = np.where((q[None, :] & np.uint64(1)) == 1, hh >> np.uint64(16), hh & np.uint64(0xFFFF))
            out[sq, h] = half >= thresh
    return out


def ln_keep_mask(seed: int, stream: int, M: int, N: int, p: float) -> np.ndarray:
    """bool [M, N]: the element-dropout mask of the fused LayerNorm kernels (csrc/train.hip
    ln_drop8): keep (m, n) iff half (n & 1) of mix24(base + m * 0x9E3779B1 + (n >> 1) *
    0x85EBCA77) >= thresh, base = fmix32(lo(seed) ^ fmix32(hi(seed) + stream * 0xC2B2AE3D))."""
    thresh = np.uint64(max(1, int(p * 65536.0 + 0.5))) if p > 0 else np.uint64(0)
    lo, hi = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    base = fmix32(lo ^ fmix32((hi + np.uint64(stream) * np.uint64(0xC2B2AE3D)) & M32))
    m = np.arange(M, dtype=np.uint64)[:, None]
    n = np.arange(N, dtype=np.uint64)[None, :]
    hh = mix24((base + m * np.uint64(0x9E3779B1) + (n >> np.uint64(1)) * np.uint64(0x85EBCA77)) & M32)
    half = np.where((n & np.uint64(1)) == 1, hh >> np.uint64(16), hh & np.uint64(0xFFFF))
    return half >= thresh
