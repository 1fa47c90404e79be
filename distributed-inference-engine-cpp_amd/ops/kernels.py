"""torch-facing wrappers around the hand-written gfx950 kernels (csrc/kernels/*.hip).

Used by the GPU numerics tests: each wrapper takes torch tensors on `cuda`, launches the native
kernel on torch's current stream through the C ABI (`capi_kernels.cpp`), and returns torch tensors.
They fail loudly (NativeError) when the native library is missing; there is no eager fallback.
"""
from __future__ import annotations

import json
from typing import Optional

import numpy as np

from .. import native


def _ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


def _stream() -> int:
    import torch

    return int(torch.cuda.current_stream().cuda_stream)


def _check(rc: int, what: str):
    if rc != 0:
        raise native.NativeError("%s launch failed (hipError %d)" % (what, rc))


def bf16_bits(t):
    """bf16 tensor -> int16 view (the kernels take raw uint16 storage)."""
    import torch

    return t.contiguous().view(torch.int16)


def split_planes(t):
    """fp32 tensor -> its split form (csrc/kernels/common.h): [2, *shape] bf16, plane 0 = hi = bf16(t),
    plane 1 = lo = bf16(t - hi) (both round to nearest even, like the device)."""
    import torch

    t = t.float()
    hi = t.to(torch.bfloat16)
    lo = (t - hi.float()).to(torch.bfloat16)
    return torch.stack([hi, lo]).contiguous()


def join_planes(p):
    """[2, ...] split planes -> fp32 (hi + lo)."""
    return p[0].float() + p[1].float()


def pack_conv_weight(w, cin_store: Optional[int] = None, npad: int = 128, split: bool = False):
    """[Cout, Cin, KH, KW] float -> [Npad][Kpad] bf16 with k = (ky*KW + kx)*Cin_store + ci.
    split: [2][Npad][Kpad] (hi plane, then lo plane)."""
    import torch

    cout, cin, kh, kw = w.shape
    cs = cin_store or cin
    K = kh * kw * cs
    Kpad = (K + 63) // 64 * 64
    Np = (cout + npad - 1) // npad * npad
    wp = torch.zeros((Np, kh, kw, cs), dtype=torch.float32, device=w.device)
    wp[:cout, :, :, :cin] = w.permute(0, 2, 3, 1).float()
    wp = wp.reshape(Np, K)
    full = torch.zeros((Np, Kpad), dtype=torch.float32, device=w.device)
    full[:, :K] = wp
    out = split_planes(full) if split else full.to(torch.bfloat16)
    return out, K, Kpad


# launch configs of the conv kernel: tile + 4 * variant (kernels.h TileCfg)
NUM_CFGS = 40  # kernels.h TileCfg (variant 7 = the 8-wave wide tile, cfg 28 only; variant 8 = skinny rows, cfg 32 only;
#               variant 9 = the four-tile 3x3 kernel, cfg 39 only)


class ConvProblem:
    """One implicit-GEMM conv problem with packed weights and preallocated outputs, re-launchable with
    any (config, split-K, fused) choice -- used by conv2d_nhwc and by tools/conv_bench.py.
    x_nhwc: [B,H,W,Cin] bf16 (split: any float dtype, converted to hi/lo planes), w: [Cout,Cin,KH,KW]
    float.  split = fp32 mode: x/res/out/out2 are split planes and the weights are packed hi + lo."""

    def __init__(self, x_nhwc, w, bias=None, stride=1, pad=0, dil=1, relu=False, res=None, out_f32=False,
                 scale2=None, shift2=None, relu2=False, max_splits=16, split=False):
        import torch

        B, H, W, Cs = x_nhwc.shape
        cout, cin, kh, kw = w.shape
        self.split = split
        self.wp, K, Kpad = pack_conv_weight(w, Cs, split=split)
        Ho = (H + 2 * pad - dil * (kh - 1) - 1) // stride + 1
        Wo = (W + 2 * pad - dil * (kw - 1) - 1) // stride + 1
        dev = x_nhwc.device

        def padded(v):
            if v is None:
                return None
            n = (v.numel() + 127) // 128 * 128
            o = torch.zeros(n, dtype=torch.float32, device=dev)
            o[: v.numel()] = v.float()
            return o

        np_ = (2,) if split else ()
        self.x = split_planes(x_nhwc) if split else x_nhwc.contiguous()
        self.res = None if res is None else (split_planes(res.reshape(B, Ho, Wo, cout)) if split else res.contiguous())
        self.bias_p, self.s2_p, self.b2_p = padded(bias), padded(scale2), padded(shift2)
        self.out_f32 = out_f32
        self.out = (torch.empty((B, Ho, Wo, cout), dtype=torch.float32, device=dev) if out_f32 else
                    torch.empty(np_ + (B, Ho, Wo, cout), dtype=torch.bfloat16, device=dev))
        self.out2 = (torch.empty(np_ + (B, Ho, Wo, cout), dtype=torch.bfloat16, device=dev)
                     if scale2 is not None else None)
        self.geom = dict(B=B, H=H, W=W, Cin=Cs, Ho=Ho, Wo=Wo, N=cout, KH=kh, KW=kw, stride=stride, pad_h=pad,
                         pad_w=pad, dil=dil, K=K, Kpad=Kpad, relu=int(relu), relu2=int(relu2))
        if split:
            self.geom.update(split=1, wplane=int(self.wp[0].numel()))
        self.zeros = torch.zeros(Kpad + 64, dtype=torch.int16, device=dev)  # zero page >= Kpad + 64
        self.geom["zeros"] = int(self.zeros.data_ptr())
        self.ws = torch.empty(max(1, max_splits) * B * Ho * Wo * cout if max_splits > 1 else 1, dtype=torch.float32,
                              device=dev)
        # fused split-K: the last split block of a tile reduces in-kernel (counters start at zero and
        # are reset by that block)
        self.counters = torch.zeros(65536, dtype=torch.int32, device=dev)
        self.flops = 2.0 * B * Ho * Wo * cout * cin * kh * kw
        self._L = native.kernels()

    def launch(self, tile=-1, splits=1, fused_splitk=True, order=0, extra=None, sk=0) -> int:
        """Launch on torch's current stream; returns the hipError code (1 = config not applicable).
        order: XCD tile order (ConvArgs::order: 0 heuristic, 1 N-fastest, 2 M-fastest).
        extra: more ConvArgs fields by geometry-JSON key (device pointers as ints), e.g. the LayerNorm
        statistics row_stats / col_sum / row_parts / stats_out and ln_eps.
        sk > 0: a stream-K launch of sk blocks (ConvArgs::sk; in-kernel reduction, splits ignored)."""
        g = dict(self.geom, splits=int(splits), order=int(order))
        g.update(extra or {})
        if sk > 0:
            bm, bn = [(128, 128), (128, 64), (64, 128), (64, 64)][tile % 4] if tile >= 0 else (64, 64)
            if self.ws.numel() < sk * 2 * bm * bn:
                return 1  # workspace too small for this P: not applicable
            g["sk"] = int(sk)
            g["ws"] = int(self.ws.data_ptr())
            g["counters"] = int(self.counters.data_ptr())
            g["counters_n"] = int(self.counters.numel())
        elif splits > 1:
            g["ws"] = int(self.ws.data_ptr())
            if fused_splitk:
                g["counters"] = int(self.counters.data_ptr())
                g["counters_n"] = int(self.counters.numel())
        return self._L.die_kern_conv(json.dumps(g).encode(), _ptr(self.x), _ptr(self.wp), _ptr(self.bias_p),
                                     _ptr(self.res), 0 if self.out_f32 else _ptr(self.out),
                                     _ptr(self.out) if self.out_f32 else 0, _ptr(self.s2_p), _ptr(self.b2_p),
                                     _ptr(self.out2), tile, _stream())

    def results(self):
        """(out, out2); split planes joined to fp32."""
        if not self.split:
            return self.out, self.out2
        out = self.out if self.out_f32 else join_planes(self.out)
        return out, None if self.out2 is None else join_planes(self.out2)


def conv2d_nhwc(x_nhwc, w, bias=None, stride=1, pad=0, dil=1, relu=False, res=None, out_f32=False,
                scale2=None, shift2=None, relu2=False, tile=-1, splits=1, fused_splitk=True, split=False):
    """Implicit-GEMM conv.  x_nhwc: [B,H,W,Cin] bf16, w: [Cout,Cin,KH,KW] float.
    Returns (out, out2) in NHWC ([B,Ho,Wo,Cout]); out is f32 if out_f32 else bf16.
    split (fp32 mode): x/res any float dtype; outputs are the fp32 values of the split planes."""
    pr = ConvProblem(x_nhwc, w, bias, stride, pad, dil, relu, res, out_f32, scale2, shift2, relu2, max_splits=splits,
                     split=split)
    rc = pr.launch(tile, splits, fused_splitk)
    if rc != 0 and tile >= 0 and rc == 1:  # hipErrorInvalidValue: config not applicable to this shape
        return None, None
    _check(rc, "conv_igemm")
    return pr.results()


def pair_permute(n_rows: int):
    """Row permutation of conv_pair weights (kernels.h pair_permute_row): physical row of logical n."""
    perm = []
    for n in range(n_rows):
        b, r = n & ~31, n & 31
        g, h, t = r >> 3, (r >> 2) & 1, r & 3
        perm.append(b + 16 * h + 4 * g + t)
    return perm


def _pack_pair_weight(w, split):
    """[N, K] float -> rows permuted by pair_permute, N padded to 128, bf16 or split planes."""
    import torch

    n, k = w.shape
    npad = (n + 127) // 128 * 128
    full = torch.zeros((npad, k), dtype=torch.float32, device=w.device)
    perm = torch.tensor(pair_permute(n), device=w.device)
    full[perm] = w.float()
    return split_planes(full) if split else full.to(torch.bfloat16)


def conv_pair(y, w1, b1, res, s2, h2, w2, b2, relu=True, relu2=True, split=False, store_x=True, store_a=False,
              shared_w=-1):
    """Fused expand + next-reduce 1x1 pair (kernels/conv_pair.hip) over rows.
    y [M, K1], w1 [N1, K1], b1 [N1], res [M, N1], s2/h2 [N1], w2 [N2, N1], b2 [N2] (float).
    Returns (x, out): x = y @ w1.T + b1 + res  [M, N1] (None unless store_x) and
    out = act(act2(x * s2 + h2) @ w2.T + b2)  [M, N2], as fp32 (split planes joined) or bf16;
    store_a: also the stored pre-activation a = act2(x * s2 + h2) [M, N1] (PairArgs::aout), as a
    third element.  shared_w: PairArgs::shared_w (-1 auto, 0 separate W1 / W2 buffers, 1 one shared buffer)."""
    import torch

    M, K1 = y.shape
    N1, N2 = w1.shape[0], w2.shape[0]
    dev = y.device
    np_ = (2,) if split else ()
    yy = _in(y, split)
    rr = _in(res, split)
    wp1 = _pack_pair_weight(w1, split)
    wp2 = _pack_pair_weight(w2, split)
    f = lambda v: v.float().contiguous()
    xo = torch.empty(np_ + (M, N1), dtype=torch.bfloat16, device=dev) if store_x else None
    out = torch.empty(np_ + (M, N2), dtype=torch.bfloat16, device=dev)
    zeros = torch.zeros(4096, dtype=torch.int16, device=dev)
    g = dict(M=M, K1=K1, N1=N1, N2=N2, relu=int(relu), relu2=int(relu2), split=int(split), zeros=int(zeros.data_ptr()),
             shared_w=int(shared_w))
    ao = torch.empty(np_ + (M, N1), dtype=torch.bfloat16, device=dev) if store_a else None
    if store_a:
        g["aout"] = int(ao.data_ptr())
    if split:
        g.update(wplane1=int(wp1[0].numel()), wplane2=int(wp2[0].numel()))
    bb1, ss2, hh2, bb2 = f(b1), f(s2), f(h2), f(b2)
    rc = native.kernels().die_kern_conv_pair(json.dumps(g).encode(), _ptr(yy), _ptr(wp1), _ptr(bb1), _ptr(rr),
                                             _ptr(xo), _ptr(ss2), _ptr(hh2), _ptr(wp2), _ptr(bb2), _ptr(out),
                                             _stream())
    _check(rc, "conv_pair")
    if store_a:
        return (None if xo is None else _out(xo, split)), _out(out, split), _out(ao, split)
    return (None if xo is None else _out(xo, split)), _out(out, split)


def _in(x, split):
    return split_planes(x) if split else x.contiguous()


def _out(y, split):
    return join_planes(y) if split else y


def input_prep(x_nchw, scale=None, shift=None, cp=4, split=False):
    import torch

    B, C, H, W = x_nchw.shape
    out = torch.empty(((2,) if split else ()) + (B, H, W, cp), dtype=torch.bfloat16, device=x_nchw.device)
    L = native.kernels()
    xin = x_nchw.contiguous().float()  # locals keep every launched-on buffer alive through the launch
    rc = L.die_kern_input_prep(_ptr(xin), _ptr(scale), _ptr(shift), _ptr(out), B, C, H, W, cp,
                               _stream(), int(split))
    _check(rc, "input_prep")
    return _out(out, split)


def pool2d_nhwc(x, k, stride, pad, is_max=True, count_include_pad=False, split=False):
    import torch

    B, H, W, C = x.shape
    Ho = (H + 2 * pad - k) // stride + 1
    Wo = (W + 2 * pad - k) // stride + 1
    y = torch.empty(((2,) if split else ()) + (B, Ho, Wo, C), dtype=torch.bfloat16, device=x.device)
    xin = _in(x, split)
    rc = native.kernels().die_kern_pool2d(_ptr(xin), _ptr(y), B, H, W, C, Ho, Wo, k, k, stride, stride, pad,
                                          pad, int(is_max), int(count_include_pad), _stream(), int(split))
    _check(rc, "pool2d")
    return _out(y, split)


def global_avgpool_nhwc(x, scale=None, shift=None, relu=False, split=False):
    import torch

    B, H, W, C = x.shape
    out = torch.empty(((2,) if split else ()) + (B, C), dtype=torch.bfloat16, device=x.device)
    out32 = torch.empty((B, C), dtype=torch.float32, device=x.device)
    xin = _in(x, split)
    rc = native.kernels().die_kern_gap(_ptr(xin), _ptr(out), _ptr(out32), _ptr(scale), _ptr(shift),
                                       int(relu), B, H * W, C, _stream(), int(split))
    _check(rc, "global_avgpool")
    return _out(out, split), out32


def affine_act(x, scale=None, shift=None, z=None, relu=False, split=False):
    import torch

    C = x.shape[-1]
    M = x.numel() // C
    y = torch.empty(((2,) if split else ()) + tuple(x.shape), dtype=torch.bfloat16, device=x.device)
    zz = None if z is None else _in(z, split)
    xin = _in(x, split)
    rc = native.kernels().die_kern_affine(_ptr(xin), _ptr(zz), _ptr(scale), _ptr(shift), int(relu), _ptr(y),
                                          M, C, _stream(), int(split))
    _check(rc, "affine_act")
    return _out(y, split)


# ---- transformer kernels (csrc/kernels/transformer.hip) ---------------------------------------------

def linear(x, w, bias=None, act=0, res=None, tile=-1, splits=1, split=False):
    """Rows GEMM on the MFMA conv kernel: x [..., K] bf16, w [N, K] float -> act(x @ w^T + bias + res).
    act: 0 none, 1 relu, 2 erf-GELU.  split: fp32 mode (fp32 result)."""
    K = x.shape[-1]
    lead = x.shape[:-1]
    M = x.numel() // K
    N = w.shape[0]
    r = None if res is None else res.reshape(M, 1, 1, N)
    out, _ = conv2d_nhwc(x.reshape(M, 1, 1, K), w.reshape(N, K, 1, 1), bias=bias, relu=act, res=r, tile=tile,
                         splits=splits, split=split)
    return None if out is None else out.reshape(*lead, N)


def layernorm(x, gamma, beta, eps=1e-5, split=False, variant=0):
    import torch

    C = x.shape[-1]
    y = torch.empty(((2,) if split else ()) + tuple(x.shape), dtype=torch.bfloat16, device=x.device)
    xin, gm, bt = _in(x, split), gamma.float().contiguous(), beta.float().contiguous()
    rc = native.kernels().die_kern_layernorm(_ptr(xin), _ptr(y), _ptr(gm), _ptr(bt), float(eps), x.numel() // C, C, _stream(),
                                             int(split), int(variant))
    _check(rc, "layernorm")
    return _out(y, split)


def tokens_assemble(patches, cls=None, pos=None, split=False):
    """patches [B, S0, C] bf16, cls [C] f32, pos [S0+1, C] f32 -> [B, S0+1, C] bf16."""
    import torch

    B, S0, C = patches.shape
    out = torch.empty(((2,) if split else ()) + (B, S0 + 1, C), dtype=torch.bfloat16, device=patches.device)
    pin = _in(patches, split)
    rc = native.kernels().die_kern_tokens(_ptr(pin), _ptr(cls), _ptr(pos), _ptr(out), B, S0, C,
                                          _stream(), int(split))
    _check(rc, "tokens_assemble")
    return _out(out, split)


def gather_rows(x, idx, split=False):
    import torch

    B, S, C = x.shape
    y = torch.empty(((2,) if split else ()) + (B, C), dtype=torch.bfloat16 if split else x.dtype, device=x.device)
    xin = _in(x, split)
    rc = native.kernels().die_kern_gather_rows(_ptr(xin), _ptr(y), B, S, int(idx), C, _stream(), int(split))
    _check(rc, "gather_rows")
    return _out(y, split)


def attention(q, k, v, heads, scale=None):
    """q/k/v: [B, S, H*D] bf16 (may be column slices of a wider tensor, row stride = stride(1)).
    Returns softmax(scale * Q K^T) V merged back to [B, S, H*D] bf16."""
    import torch

    B, S, C = q.shape
    D = C // heads
    for t in (q, k, v):
        assert t.stride(2) == 1 and t.stride(0) == S * t.stride(1), "rows must be [B*S][ld] with unit column stride"
    out = torch.empty((B, S, C), dtype=torch.bfloat16, device=q.device)
    sc = float(scale if scale is not None else 1.0 / np.sqrt(D))
    rc = native.kernels().die_kern_attention(_ptr(q), _ptr(k), _ptr(v), _ptr(out), B, S, heads, D, q.stride(1),
                                             k.stride(1), v.stride(1), C, sc, _stream(), 0)
    _check(rc, "attention")
    return out


def set_attention_variant(v):
    """Process-wide streaming-attention variant (kernels.h set_attention_variant): 0 = K/V staged one
    tile ahead (default), 1 = two tiles ahead."""
    native.kernels().die_kern_set_attention_variant(int(v))


def attention_qkv_split(qkv, heads, scale=None):
    """fp32 mode: qkv [B, S, 3*C] float (Q | K | V columns) -> fp32 [B, S, C] through the split kernel
    (planes of the packed QKV rows, like the engine's fused QKV GEMM output)."""
    import torch

    B, S, C3 = qkv.shape
    C = C3 // 3
    D = C // heads
    planes = split_planes(qkv)  # [2, B, S, 3C]
    out = torch.empty((2, B, S, C), dtype=torch.bfloat16, device=qkv.device)
    sc = float(scale if scale is not None else 1.0 / np.sqrt(D))
    base = _ptr(planes)
    rc = native.kernels().die_kern_attention(base, base + 2 * C, base + 4 * C, _ptr(out), B, S, heads, D, C3, C3, C3,
                                             C, sc, _stream(), 1)
    _check(rc, "attention (split)")
    return join_planes(out)


# ---- device JSON decode (csrc/kernels/decode.hip) ---------------------------------------------------

def decode_json_numbers(texts, numel, text_cap=None, slot_order=None, packed=False):
    """Decode number-list texts (bytes, the inside of a JSON array; None = skipped sample) on the GPU.
    slot_order: optional permutation; sample i's text is then placed in arena slot slot_order[i]
    and located through the per-sample offset table (the engine's staged-upload layout).
    packed: upload every text that packs (core/textpack.h) 4-bit packed, the worker's default (the
    nibble-level kernels decode those; the rest stays raw).
    Returns (values [B, numel] f32, status [B] int32, ntok [B] int32) as torch tensors."""
    import torch

    B = len(texts)
    if text_cap is None:
        text_cap = max(4096, max(len(t) for t in texts if t is not None) + 64)
        text_cap = (text_cap + 4095) // 4096 * 4096
    slots = list(range(B)) if slot_order is None else list(slot_order)
    nslots = max(slots) + 1 if slots else 1
    host = np.zeros(nslots * text_cap, np.uint8)
    lens = np.full(B, -1, np.int64)
    offs = np.zeros(B, np.int64)
    for i, t in enumerate(texts):
        offs[i] = slots[i] * text_cap
        if t is None:
            continue
        assert len(t) <= text_cap
        host[offs[i]:offs[i] + len(t)] = np.frombuffer(t, np.uint8)
        lens[i] = len(t)
    L = native.kernels()
    d_text = torch.from_numpy(host).cuda()
    d_lens = torch.from_numpy(lens).cuda()
    d_offs = torch.from_numpy(offs).cuda() if slot_order is not None else None
    out = torch.full((B, numel), float("nan"), dtype=torch.float32, device="cuda")
    status = torch.full((B,), -7, dtype=torch.int32, device="cuda")
    ntok = torch.zeros(B, dtype=torch.int32, device="cuda")
    scratch = torch.empty(int(L.die_decode_scratch_bytes(B, text_cap)), dtype=torch.uint8, device="cuda")
    if packed:
        hp = np.zeros(nslots * text_cap // 2, np.uint8)
        poffs = np.full(B, -1, np.int64)
        for i, t in enumerate(texts):
            pk = native.pack_nibbles(t) if t is not None else None
            if pk is not None:
                poffs[i] = slots[i] * (text_cap // 2)
                hp[poffs[i]:poffs[i] + len(pk)] = np.frombuffer(pk, np.uint8)
        d_packed = torch.from_numpy(hp).cuda()
        d_poffs = torch.from_numpy(poffs).cuda()
        if d_offs is None:
            d_offs = torch.from_numpy(offs).cuda()
        rc = L.die_kern_decode_packed(_ptr(d_text), _ptr(d_offs), _ptr(d_packed), _ptr(d_poffs), text_cap, _ptr(d_lens),
                                      B, _ptr(out), numel, _ptr(status), _ptr(ntok), _ptr(scratch), _stream())
    else:
        rc = L.die_kern_decode(_ptr(d_text), _ptr(d_offs), text_cap, _ptr(d_lens), B, _ptr(out), numel, _ptr(status),
                               _ptr(ntok), _ptr(scratch), _stream())
    _check(rc, "decode_json_numbers")
    return out, status, ntok


def pack_stem_weight(w, split=False):
    """[64, C<=4, 7, 7] float -> [64][224] bf16 with k = ky*32 + kx*4 + c (kx padded to 8)
    (split: [2][64][224] hi, lo planes)."""
    import torch

    co, ci = w.shape[:2]
    wp = torch.zeros((co, 7, 8, 4), dtype=torch.float32, device=w.device)
    wp[:, :, :7, :ci] = w.float().permute(0, 2, 3, 1)
    wp = wp.reshape(co, 224)
    return split_planes(wp) if split else wp.to(torch.bfloat16).contiguous()


def conv_stem7x7(x_nhwc4, w, bias, relu=True, split=False):
    """ResNet stem on the LDS-patch kernel: x [B,H,W,4] bf16, w [64,C,7,7] -> [B,Ho,Wo,64] bf16.
    split (fp32 mode): x any float dtype, fp32 result."""
    import torch

    B, H, W, C = x_nhwc4.shape
    assert C == 4 and w.shape[0] == 64
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    out = torch.empty(((2,) if split else ()) + (B, Ho, Wo, 64), dtype=torch.bfloat16, device=x_nhwc4.device)
    b = bias.float().contiguous()
    xin, wp = _in(x_nhwc4, split), pack_stem_weight(w, split)
    rc = native.kernels().die_kern_stem(_ptr(xin), _ptr(wp), _ptr(b), _ptr(out),
                                        B, H, W, Ho, Wo, int(relu), _stream(), int(split))
    _check(rc, "conv_stem7x7")
    return _out(out, split)


def conv_stem7x7_nchw(x_nchw, w, bias, scale=None, shift=None, relu=True, split=False, max_blocks=0):
    """Persistent fused stem: x [B,C<=4,H,W] fp32 NCHW (the graph input, no input_prep pass), the
    per-channel input affine x*scale+shift applied on load, w [64,C,7,7] -> [B,Ho,Wo,64] (bf16, or the
    fp32 values of the split planes).  max_blocks > 0 caps the grid (tests: several tiles per block)."""
    import torch

    B, C, H, W = x_nchw.shape
    assert C <= 4 and w.shape[0] == 64
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    out = torch.empty(((2,) if split else ()) + (B, Ho, Wo, 64), dtype=torch.bfloat16, device=x_nchw.device)
    xin = x_nchw.float().contiguous()
    b = bias.float().contiguous()
    sc = None if scale is None else scale.float().contiguous()
    sh = None if shift is None else shift.float().contiguous()
    wp = pack_stem_weight(w, split)
    rc = native.kernels().die_kern_stem_nchw(_ptr(xin), C, _ptr(sc), _ptr(sh), _ptr(wp), _ptr(b), _ptr(out),
                                             B, H, W, Ho, Wo, int(relu), _stream(), int(split), int(max_blocks))
    _check(rc, "conv_stem7x7_nchw")
    return _out(out, split)


# ---- grouped conv / row softmax (csrc/kernels/gconv.hip, transformer.hip) ---------------------------

def grouped_conv(x_nhwc, w, bias=None, stride=1, pads=(0, 0, 0, 0), groups=1, clip=None, relu=False, split=False):
    """x [B,H,W,Cin] (bf16, or any float dtype with split), w [Cout, Cin/groups, k, k] float,
    pads [top, left, bottom, right] -> [B,Ho,Wo,Cout] (fp32 values of the split planes when split)."""
    import torch

    B, H, W, Cin = x_nhwc.shape
    Cout, cpg, KH, KW = w.shape
    Ho = (H + pads[0] + pads[2] - KH) // stride + 1
    Wo = (W + pads[1] + pads[3] - KW) // stride + 1
    xin = _in(x_nhwc, split) if split else x_nhwc.to(torch.bfloat16).contiguous()
    wp = w.float().permute(0, 2, 3, 1).contiguous()
    bp = None if bias is None else bias.float().contiguous()
    out = torch.empty(((2,) if split else ()) + (B, Ho, Wo, Cout), dtype=torch.bfloat16, device=x_nhwc.device)
    act = 3 if clip is not None else (1 if relu else 0)
    lo, hi = clip if clip is not None else (0.0, 0.0)
    geom = dict(B=B, H=H, W=W, Cin=Cin, Ho=Ho, Wo=Wo, Cout=Cout, groups=groups, KH=KH, KW=KW, stride=stride,
                pad_h=pads[0], pad_w=pads[1], act=act, clip_lo=float(lo), clip_hi=float(hi), split=int(split))
    rc = native.kernels().die_kern_gconv(json.dumps(geom).encode(), _ptr(xin), _ptr(wp), _ptr(bp), _ptr(out), _stream())
    _check(rc, "grouped_conv")
    return _out(out, split)


def softmax_rows(x, split=False):
    """x [rows, C] float -> (softmax stored bf16/split -> fp32 values, softmax fp32)."""
    import torch

    rows, C = x.shape
    xin = _in(x, split) if split else x.to(torch.bfloat16).contiguous()
    y = torch.empty(((2,) if split else ()) + (rows, C), dtype=torch.bfloat16, device=x.device)
    yf = torch.empty((rows, C), dtype=torch.float32, device=x.device)
    rc = native.kernels().die_kern_softmax(_ptr(xin), _ptr(y), _ptr(yf), rows, C, _stream(), int(split))
    _check(rc, "softmax_rows")
    return (join_planes(y) if split else y.float()), yf
