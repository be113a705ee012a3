"""BERT-large (SQuAD head) for the ``bert_large`` bench model (random-init).

Public BERT-large architecture: vocab 30522, hidden 1024, 24 layers, 16
heads, FFN 4096, GELU, post-LN, max 512 positions, 2 token types; the
question-answering head maps every token to (start, end) logits.  Weights are
random (seeded, std 0.02 as in BERT's initializer) — there is no checkpoint
on the box.

Compute layout for MI355X: bf16 everywhere, fused QKV projection (one
[3H, H] GEMM per layer instead of three), attention as ONE hand-written HIP
kernel (K12, csrc/kernels/bert.hip) that reads Q/K/V straight from the QKV
GEMM's output (computed without its bias, which K12 applies), applies the
key-padding mask and writes the [tokens, hidden] layout the output projection reads (torch SDPA is the fallback for sequences
over 384 or off the GPU), the projections on the hand-written K18 GEMM
(csrc/kernels/gemm_tiles.hip) at the token counts where it beat hipBLASLt
(gemm_route: up to 768 tokens, the attention-out projection to 3,072; the
N = 1024 projections split over K into fp32 slabs that the LayerNorm kernel
sums) and on hipBLASLt above, the GELU
in the FFN-up GEMM's epilogue and every
residual add + LayerNorm as ONE hand-written HIP kernel (K11,
csrc/kernels/bert.hip), as is the embedding sum + LayerNorm.  The serving wrapper captures one HIP graph per
batch bucket.
"""

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

VOCAB = 30522
HIDDEN = 1024
LAYERS = 24
HEADS = 16
FFN = 4096
MAX_POS = 512
TYPES = 2


# fused paths on the GPU (bf16 CUDA tensors); TC_BERT_FUSED=0 runs plain torch ops
FUSED = os.environ.get("TC_BERT_FUSED", "1") != "0"
# Who runs the four projection GEMMs: "auto" = the measured routing table
# below (our K18 where it beat hipBLASLt, the library elsewhere), "ours" =
# the hand-written kernels everywhere (K18 for small / mid token counts, K17
# above), "lib" = hipBLASLt everywhere.
GEMM = os.environ.get("TC_BERT_GEMM", "auto")

# Measured routing (tools/gemm_sweep.py on MI355X, profiles/r6_gemm/: each
# arm in a HIP graph over weight copies past the Infinity Cache, the N = 1024
# projections timed together with the residual add + LayerNorm that follows
# them).  Per projection: (largest token count, route), first match wins, the
# last entry covers every larger count; route = ("k18", cfg, splits) --
# splits > 1 leaves fp32 partial slabs that K11p sums into the LayerNorm --
# ("k17",) / ("k17", 0) (K17, claimed / static tile lists) or ("lib",)
# (hipBLASLt: where it measured faster).
INF = 1 << 30
GEMM_ROUTES = {
    "qkv": [(384, ("k18", 6, 1)), (768, ("k18", 3, 1)), (4608, ("lib",)), (6144, ("k17", 0)), (INF, ("lib",))],
    "out": [(384, ("k18", 9, 1)), (768, ("k18", 6, 1)), (1536, ("k18", 0, 1)), (3072, ("k18", 3, 1)),
            (INF, ("lib",))],
    "ffn_up": [(384, ("k18", 1, 1)), (768, ("k18", 3, 1)), (INF, ("lib",))],
    "ffn_down": [(384, ("k18", 6, 2)), (768, ("k18", 7, 2)), (1536, ("k18", 2, 2)), (INF, ("lib",))],
}
# the fp32-parity model's bf16x3 projections (K tripled, fp32 out, erf GELU;
# tools/gemm_sweep.py --x3, whose library arm adds the bias and the GELU as
# separate ops, as torch.mm must)
#
# Past 3,072 tokens every x3 projection stays on K17 even where the library
# measured faster (QKV 188 vs 216 us, FFN-down 281 vs 312 us at 12,288
# tokens): served with two instances (two streams), the fp32 model stalled
# twice at c256 with one instance thread waiting in hipStreamSynchronize
# forever (profiles/r6_bert_fp32/); the library's large fp32-output GEMMs were
# the only kernels of that graph not ours, so they are kept off it.
GEMM_ROUTES_X3 = {
    "qkv": [(384, ("k18", 6, 1)), (3072, ("lib",)), (INF, ("k17", 0))],
    "out": [(384, ("k18", 6, 2)), (768, ("k18", 2, 2)), (1536, ("k18", 3, 2)), (3072, ("k18", 3, 1)),
            (INF, ("k17", 0))],
    "ffn_up": [(384, ("k18", 1, 1)), (768, ("k18", 3, 1)), (1536, ("lib",)), (INF, ("k17", 0))],
    "ffn_down": [(384, ("k18", 7, 4)), (768, ("k18", 3, 4)), (1536, ("k18", 3, 2)), (3072, ("lib",)),
                 (INF, ("k17", 0))],
}
OURS_FROM_K17 = 3072  # "ours" mode where the table says lib: K17 from this many tokens, K18 cfg 3 below


def _route(table, name, M, mode):
    if mode == "lib" or name is None:
        return ("lib",)
    for top, route in table[name]:
        if M <= top:
            break
    if route[0] == "lib" and mode == "ours":
        return ("k17",) if M >= OURS_FROM_K17 else ("k18", 3, 1)
    return route


def gemm_route(name, M, mode=None):
    """The kernel that runs bf16 projection ``name`` at ``M`` tokens: ("lib",),
    ("k17"[, dyn]) or ("k18", cfg, splits).  mode (default TC_BERT_GEMM): auto
    = the table, ours = the table with every library entry replaced by K17 /
    K18, lib = hipBLASLt everywhere."""
    return _route(GEMM_ROUTES, name, M, mode or GEMM)


def gemm_route_x3(name, M, mode=None):
    """The kernel of the fp32-parity (bf16x3) projection ``name`` at ``M`` tokens."""
    return _route(GEMM_ROUTES_X3, name, M, mode or GEMM)


def _bias_f32(lin, dev):
    b = getattr(lin, "bias_f32", None)
    if b is None or b.device != dev:
        b = lin.bias_f32 = lin.bias.detach().float().contiguous()
    return b


def _ours_ok(x2, lin):
    return (FUSED and x2.is_cuda and x2.dtype == torch.bfloat16 and lin.weight.dtype == torch.bfloat16
            and x2.stride(1) == 1 and x2.stride(0) % 8 == 0 and x2.data_ptr() % 16 == 0 and lin.weight.is_contiguous())


def _k17_launch(route, *args, **kw):
    """K17 with the route's scheduling: ("k17",) the TCAMD_K17_DYN default,
    ("k17", 0) static tile lists (read at launch, so a captured graph keeps it)."""
    from triton_client_amd.ops import hip

    if len(route) > 1:
        with hip.knob(TCAMD_K17_DYN=int(route[1])):
            hip.k17_gemm(*args, **kw)
    else:
        hip.k17_gemm(*args, **kw)


def _k17(x2, lin, epilogue, route=("k17",)):
    M, K = x2.shape
    N = lin.weight.shape[0]
    out = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
    bias = None if epilogue == "none" else _bias_f32(lin, x2.device)
    _k17_launch(route, x2.data_ptr(), lin.weight.data_ptr(), None if bias is None else bias.data_ptr(),
                out.data_ptr(), M, N, K, x2.stride(0), lin.weight.stride(0), N, epilogue=epilogue,
                stream=torch.cuda.current_stream(x2.device).cuda_stream)
    return out


def _k18(x2, lin, epilogue, cfg, splits=1):
    """K18 (csrc/kernels/gemm_tiles.hip); splits > 1: fp32 partial slabs
    [splits, M, N] (no epilogue), for K11p to sum."""
    from triton_client_amd.ops import hip

    M, K = x2.shape
    N = lin.weight.shape[0]
    st = torch.cuda.current_stream(x2.device).cuda_stream
    if splits > 1:
        out = torch.empty(splits, M, N, device=x2.device, dtype=torch.float32)
        hip.k18_gemm(x2.data_ptr(), lin.weight.data_ptr(), None, out.data_ptr(), M, N, K, x2.stride(0),
                     lin.weight.stride(0), N, out_f32=True, cfg=cfg, splits=splits, split_stride=M * N, stream=st)
        return out
    out = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
    bias = None if epilogue == "none" else _bias_f32(lin, x2.device)
    hip.k18_gemm(x2.data_ptr(), lin.weight.data_ptr(), None if bias is None else bias.data_ptr(), out.data_ptr(), M,
                 N, K, x2.stride(0), lin.weight.stride(0), N, epilogue=epilogue, cfg=cfg, stream=st)
    return out


def _route_ok(route, M, N, K):
    """The shape constraints of the routed kernel (else the library runs it)."""
    if route[0] == "k17":
        return N % 256 == 0 and K % 32 == 0
    if route[0] == "k18":
        from triton_client_amd.ops import hip

        tn = hip.k18_cfg(route[1])[1]
        return N % tn == 0 and K % (64 * route[2]) == 0
    return False


class _Parts:
    """A split-K projection's fp32 partial slabs [splits, tokens, N] (no bias)."""

    def __init__(self, slabs):
        self.slabs = slabs


class _X3:
    """An fp32 activation [..., K] that exists only as its bf16x3 GEMM operand
    xc [rows, 3K] = [hi | hi | lo] (K12x writes the attention output so)."""

    def __init__(self, xc, shape):
        self.xc = xc
        self.shape = shape


def _x3_operand(x):
    """The bf16x3 operand a producer already wrote for ``x`` (K12x's _X3, or
    the ``_x3`` a K11p LayerNorm attaches to its fp32 output), else None."""
    return x.xc if isinstance(x, _X3) else getattr(x, "_x3", None)


def _proj(x, lin, epilogue="bias", name=None, allow_split=False, x3_out=False):
    """lin(x) (epilogue "bias"), gelu(lin(x)) ("bias_gelu") or x @ W^T ("none").
    On the GPU in bf16 the routing table picks K18 / K17 (the hand-written
    gfx950 GEMMs) or hipBLASLt per projection and token count (gemm_route).
    With ``allow_split`` a split-K route returns its fp32 partial slabs
    [splits, tokens, N] as _Parts (the caller's K11p sums them with the bias).
    ``x3_out`` (fp32-parity FFN-up): a K17 route writes the GELU output as the
    next projection's bf16x3 operand and this returns it as an _X3."""
    n = lin.weight.shape[0]
    xc = _x3_operand(x)
    if xc is not None and getattr(lin, "w3", None) is not None:
        return _x3_result(_mm_x3(None, lin, epilogue, name, allow_split, xc=xc, x3_out=x3_out), x, n)
    x2 = x.reshape(-1, x.shape[-1])
    if name is not None and _ours_ok(x2, lin):
        route = gemm_route(name, x2.shape[0])
        if _route_ok(route, x2.shape[0], n, x2.shape[1]):
            if route[0] == "k17":
                return _k17(x2, lin, epilogue, route).view(*x.shape[:-1], n)
            splits = route[2] if allow_split and epilogue == "bias" else 1
            y = _k18(x2, lin, epilogue, route[1], splits)
            return _Parts(y) if splits > 1 else y.view(*x.shape[:-1], n)
    if getattr(lin, "w3", None) is not None and x2.is_cuda and x2.dtype == torch.float32:
        return _x3_result(_mm_x3(x2, lin, epilogue, name, allow_split, x3_out=x3_out), x, n)
    if epilogue == "none":
        return torch.mm(x2, lin.weight.t()).view(*x.shape[:-1], n)
    if epilogue == "bias_gelu":
        return _linear_gelu(x, lin)
    return lin(x)


def _x3_result(y, x, n):
    """_mm_x3's result in the caller's shape [..., n] (split slabs as they are)."""
    if isinstance(y, _Parts):
        return y
    if isinstance(y, _X3):
        y.shape = (*x.shape[:-1], n)
        return y
    return y.view(*x.shape[:-1], n)


def _mm_x3(x2, lin, epilogue="none", name=None, allow_split=False, xc=None, x3_out=False):
    """fp32-parity projection: x2 fp32 [M, K] against w3 = [W_hi | W_lo | W_hi]
    bf16 [N, 3K] as ONE bf16 GEMM over [x_hi | x_hi | x_lo] (csrc/kernels/bert.hip
    x3_cat): x_hi W_hi + x_hi W_lo + x_lo W_hi, fp32 accumulate and output,
    ~1e-5 of an fp32 GEMM.  The GEMM is K18 / K17 (gemm_route_x3) with the
    bias and the erf GELU in its epilogue, or a split-K route's fp32 slabs
    (_Parts) for K11p; torch.mm with TC_BERT_GEMM=lib.  ``xc``: the operand a
    producer (K11p, K12x) already wrote; then x2 is not read and no x3_cat runs."""
    from triton_client_amd.ops import hip

    w3 = lin.w3
    N = w3.shape[0]
    if xc is None:
        M, K = x2.shape
        st = torch.cuda.current_stream(x2.device).cuda_stream
        xc = torch.empty(M, 3 * K, device=x2.device, dtype=torch.bfloat16)
        hip.x3_cat(x2.contiguous().data_ptr(), xc.data_ptr(), M, K, stream=st)
    else:
        M, K = xc.shape[0], xc.shape[1] // 3
        st = torch.cuda.current_stream(xc.device).cuda_stream
    x2 = xc
    route = gemm_route_x3(name, M)
    if route[0] != "lib" and FUSED and _route_ok(route, M, N, 3 * K):
        epi = "bias_gelu_erf" if epilogue == "bias_gelu" else epilogue
        bias = None if epi == "none" else lin.bias.detach()
        if route[0] == "k18" and route[2] > 1 and allow_split and epilogue == "bias":
            out = torch.empty(route[2], M, N, device=x2.device, dtype=torch.float32)
            hip.k18_gemm(xc.data_ptr(), w3.data_ptr(), None, out.data_ptr(), M, N, 3 * K, 3 * K, 3 * K, N,
                         out_f32=True, cfg=route[1], splits=route[2], split_stride=M * N, stream=st)
            return _Parts(out)
        bp = None if bias is None else bias.data_ptr()
        if route[0] == "k17" and x3_out and epi == "bias_gelu_erf":
            out3 = torch.empty(M, 3 * N, device=x2.device, dtype=torch.bfloat16)
            _k17_launch(route, xc.data_ptr(), w3.data_ptr(), bp, out3.data_ptr(), M, N, 3 * K, 3 * K, 3 * K, 3 * N,
                        epilogue="bias_gelu_erf_x3", out_f32=False, stream=st)
            return _X3(out3, (M, N))
        out = torch.empty(M, N, device=x2.device, dtype=torch.float32)
        if route[0] == "k17":
            _k17_launch(route, xc.data_ptr(), w3.data_ptr(), bp, out.data_ptr(), M, N, 3 * K, 3 * K, 3 * K, N,
                        epilogue=epi, out_f32=True, stream=st)
        else:
            hip.k18_gemm(xc.data_ptr(), w3.data_ptr(), bp, out.data_ptr(), M, N, 3 * K, 3 * K, 3 * K, N,
                         epilogue=epi, out_f32=True, cfg=route[1], stream=st)
        return out
    y = torch.mm(xc, w3.t(), out_dtype=torch.float32)
    if epilogue != "none":
        y += lin.bias
    if epilogue == "bias_gelu":
        y = F.gelu(y)
    return y


def prepare_x3(model):
    """fp32-parity mode of an fp32 model: every projection of every layer gets
    its bf16x3 weight w3 = [W_hi | W_lo | W_hi] (the fp32 weights stay for the
    reference path); forward() on fp32 CUDA activations then runs those GEMMs
    on the bf16 MFMA (3x the bf16 work instead of the 16x of f32-input MFMA)
    and everything else (LayerNorm, GELU, softmax attention) in fp32."""
    with torch.no_grad():
        for layer in model.layers:
            for lin in (layer.qkv, layer.out, layer.ffn1, layer.ffn2):
                w = lin.weight.float()
                hi = w.to(torch.bfloat16)
                lo = (w - hi.float()).to(torch.bfloat16)
                lin.w3 = torch.cat([hi, lo, hi], dim=1).contiguous()
    model.precision = "fp32"
    return model


def _proj_add_ln(x, a, lin, ln, name):
    """LayerNorm(x + lin(a)): the attention-out / FFN-down projection and the
    residual add + LayerNorm behind it.  A split-K route hands its fp32
    partial slabs to K11p, which sums them with the bias and the residual on
    its way into the LayerNorm (no reduce launch, no bf16 y)."""
    y = _proj(a, lin, "bias", name=name, allow_split=True)
    if isinstance(y, _Parts):
        from triton_client_amd.ops import hip

        p = y.slabs
        out = torch.empty_like(x)
        rows, H = p.shape[1], p.shape[2]
        assert x.is_contiguous() and x.numel() == rows * H
        f32 = x.dtype == torch.float32
        bias = lin.bias.detach() if f32 else _bias_f32(lin, x.device)
        xc = _x3_buffer(x, lin, rows, H)
        hip.add_layernorm_parts(x.data_ptr(), p.data_ptr(), p.shape[0], rows * H, bias.data_ptr(),
                                ln.weight.data_ptr(), ln.bias.data_ptr(), out.data_ptr(), rows, H, ln.eps, f32=f32,
                                stream=torch.cuda.current_stream(x.device).cuda_stream,
                                out3=None if xc is None else xc.data_ptr())
        if xc is not None:
            out._x3 = xc
        return out
    return _add_ln(x, y, ln, x3=getattr(lin, "w3", None) is not None)


def _x3_buffer(x, lin, rows, H):
    """The bf16x3 operand buffer a fp32-parity LayerNorm fills beside its fp32
    output (the next projection's input: no x3_cat pass), or None."""
    if x.dtype != torch.float32 or getattr(lin, "w3", None) is None:
        return None
    return torch.empty(rows, 3 * H, device=x.device, dtype=torch.bfloat16)


def _add_ln(x, y, ln, x3=False):
    """LayerNorm(x + y): K11 on the GPU (K11p's fp32 form for the fp32-parity
    model: y as its one partial slab; with ``x3`` it also writes the next
    projection's bf16x3 operand, attached as ``out._x3``), torch ops elsewhere."""
    if (FUSED and x.is_cuda and x.dtype == torch.float32 and y.dtype == torch.float32 and x.is_contiguous()
            and y.is_contiguous() and x.shape[-1] in (512, 1024, 2048, 4096)):
        from triton_client_amd.ops import hip

        out = torch.empty_like(x)
        rows, H = x.numel() // x.shape[-1], x.shape[-1]
        xc = torch.empty(rows, 3 * H, device=x.device, dtype=torch.bfloat16) if x3 else None
        hip.add_layernorm_parts(x.data_ptr(), y.data_ptr(), 1, rows * H, None, ln.weight.data_ptr(),
                                ln.bias.data_ptr(), out.data_ptr(), rows, H, ln.eps, f32=True,
                                stream=torch.cuda.current_stream(x.device).cuda_stream,
                                out3=None if xc is None else xc.data_ptr())
        if xc is not None:
            out._x3 = xc
        return out
    if FUSED and x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and y.is_contiguous():
        from triton_client_amd.ops import hip

        out = torch.empty_like(x)
        hip.add_layernorm(x.data_ptr(), y.data_ptr(), ln.weight.data_ptr(), ln.bias.data_ptr(), out.data_ptr(),
                          x.numel() // x.shape[-1], x.shape[-1], ln.eps,
                          stream=torch.cuda.current_stream(x.device).cuda_stream)
        return out
    return ln(x + y)


def _linear_gelu(x, lin):
    """gelu(lin(x)); on the GPU the GELU runs in the GEMM epilogue."""
    if FUSED and x.is_cuda:
        y = torch._addmm_activation(lin.bias, x.reshape(-1, x.shape[-1]), lin.weight.t(), use_gelu=True)
        return y.view(*x.shape[:-1], y.shape[-1])
    return F.gelu(lin(x))


def _k12_ok(x, s):
    """K12 takes this activation: bf16 on the GPU, s % 64 == 0, s <= 384."""
    if not (FUSED and x.is_cuda and x.dtype == torch.bfloat16 and s % 64 == 0 and x.is_contiguous()):
        return False
    from triton_client_amd.ops import hip

    return s <= hip.ATTENTION_MAX_SEQ


def _attention(qkv, b, s, mask_i32, bias, qkv_bias=None, x3_out=False):
    """Multi-head attention over the QKV projection [b, s, 3H]: K12 on the GPU
    (bf16), K12x (fp32-parity; mask_i32: int32 [b, s] key-padding mask or
    None), SDPA elsewhere.  ``x3_out`` (fp32-parity model): K12x writes the
    out projection's bf16x3 operand and this returns it as an _X3.
    qkv_bias: the projection's bias when ``qkv`` was computed without it."""
    if _k12_ok(qkv, s):
        from triton_client_amd.ops import hip

        out = torch.empty(b, s, HIDDEN, device=qkv.device, dtype=qkv.dtype)
        hip.attention(qkv.data_ptr(), None if mask_i32 is None else mask_i32.data_ptr(), out.data_ptr(), b, s,
                      HEADS, 1.0 / math.sqrt(HIDDEN // HEADS), stream=torch.cuda.current_stream(qkv.device).cuda_stream,
                      bias=None if qkv_bias is None else qkv_bias.data_ptr())
        return out
    if qkv_bias is not None:
        qkv = qkv + qkv_bias
    if FUSED and qkv.is_cuda and qkv.dtype == torch.float32 and s % 64 == 0 and qkv.is_contiguous():
        # fp32-parity mode: K12x (bf16x3 products, fp32 softmax) instead of fp32 SDPA
        from triton_client_amd.ops import hip

        if x3_out:
            out = torch.empty(b * s, 3 * HIDDEN, device=qkv.device, dtype=torch.bfloat16)
        else:
            out = torch.empty(b, s, HIDDEN, device=qkv.device, dtype=torch.float32)
        hip.attention_f32(qkv.data_ptr(), None if mask_i32 is None else mask_i32.data_ptr(), out.data_ptr(), b, s,
                          HEADS, 1.0 / math.sqrt(HIDDEN // HEADS),
                          stream=torch.cuda.current_stream(qkv.device).cuda_stream, x3=x3_out)
        return _X3(out, (b, s, HIDDEN)) if x3_out else out
    q, k, v = qkv.view(b, s, 3, HEADS, HIDDEN // HEADS).permute(2, 0, 3, 1, 4)
    a = F.scaled_dot_product_attention(q, k, v, attn_mask=bias)
    return a.transpose(1, 2).reshape(b, s, HIDDEN)


def _qa_head(x, qa):
    """(start, end) fp32 logits [b, s]: the QA head kernel (csrc/kernels/bert.hip qa_head) on the GPU
    (one launch instead of an N = 2 library GEMM, a cast and two strided
    copies), the Linear elsewhere."""
    b, s, H = x.shape
    if FUSED and x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.is_contiguous() and \
            qa.weight.dtype == x.dtype and H % 512 == 0:
        from triton_client_amd.ops import hip

        bias = getattr(qa, "bias_f32", None)
        if bias is None or bias.device != x.device:
            bias = qa.bias_f32 = qa.bias.detach().float().contiguous()
        out = torch.empty(2, b, s, device=x.device, dtype=torch.float32)
        hip.qa_head(x.data_ptr(), qa.weight.data_ptr(), bias.data_ptr(), out[0].data_ptr(), out[1].data_ptr(), b * s, H,
                    f32=x.dtype == torch.float32, stream=torch.cuda.current_stream(x.device).cuda_stream)
        return out[0], out[1]
    logits = qa(x).float()
    return logits[..., 0], logits[..., 1]


class _Layer(nn.Module):
    def __init__(self):
        super().__init__()
        self.qkv = nn.Linear(HIDDEN, 3 * HIDDEN)
        self.out = nn.Linear(HIDDEN, HIDDEN)
        self.ln1 = nn.LayerNorm(HIDDEN, eps=1e-12)
        self.ffn1 = nn.Linear(HIDDEN, FFN)
        self.ffn2 = nn.Linear(FFN, HIDDEN)
        self.ln2 = nn.LayerNorm(HIDDEN, eps=1e-12)

    def forward(self, x, bias, mask_i32=None):
        b, s, _ = x.shape
        if _k12_ok(x, s):
            # plain GEMM (no bias epilogue: 152 vs 171 us at bs64 x 384,
            # profiles/r3_bert_gemm_layout.log); K12 applies the bias
            qkv = _proj(x, self.qkv, "none", name="qkv")
            a = _attention(qkv, b, s, mask_i32, bias, qkv_bias=self.qkv.bias)
        else:
            a = _attention(_proj(x, self.qkv, name="qkv"), b, s, mask_i32, bias,
                           x3_out=getattr(self.out, "w3", None) is not None and x.is_cuda)
        x = _proj_add_ln(x, a, self.out, self.ln1, "out")
        return _proj_add_ln(x, _proj(x, self.ffn1, "bias_gelu", name="ffn_up", x3_out=True), self.ffn2, self.ln2,
                            "ffn_down")


class BertLargeQA(nn.Module):
    def __init__(self, layers=LAYERS):
        super().__init__()
        self.word = nn.Embedding(VOCAB, HIDDEN)
        self.pos = nn.Embedding(MAX_POS, HIDDEN)
        self.tok_type = nn.Embedding(TYPES, HIDDEN)
        self.ln = nn.LayerNorm(HIDDEN, eps=1e-12)
        self.layers = nn.ModuleList(_Layer() for _ in range(layers))
        self.qa = nn.Linear(HIDDEN, 2)

    def _embed(self, input_ids, token_type_ids):
        """LayerNorm(word + position + token-type embeddings): one HIP launch on
        the GPU (csrc/kernels/bert.hip embed_layernorm), torch ops elsewhere."""
        b, s = input_ids.shape
        w = self.word.weight
        if FUSED and w.is_cuda and w.dtype == torch.bfloat16 and s <= MAX_POS:
            from triton_client_amd.ops import hip

            ids = input_ids.to(torch.int64).contiguous()
            tt = token_type_ids.to(torch.int64).contiguous()
            out = torch.empty(b, s, HIDDEN, device=w.device, dtype=w.dtype)
            hip.embed_layernorm(ids.data_ptr(), tt.data_ptr(), w.data_ptr(), self.pos.weight.data_ptr(),
                                self.tok_type.weight.data_ptr(), self.ln.weight.data_ptr(), self.ln.bias.data_ptr(),
                                out.data_ptr(), b * s, s, HIDDEN, VOCAB, TYPES, self.ln.eps,
                                stream=torch.cuda.current_stream(w.device).cuda_stream)
            return out
        pos = torch.arange(s, device=input_ids.device)
        return self.ln(self.word(input_ids) + self.pos(pos)[None] + self.tok_type(token_type_ids))

    def forward(self, input_ids, attention_mask, token_type_ids, dense=False):
        """dense=True: the caller guarantees attention_mask is all ones, so
        attention runs without a bias (torch-ROCm's unmasked fused kernel is
        ~1.8x faster at bs64 x 384, tools/attn_probe.py)."""
        b, s = input_ids.shape
        x = self._embed(input_ids, token_type_ids)
        # additive key-padding mask [b, 1, 1, s] in the compute dtype
        bias = None if dense else ((1.0 - attention_mask[:, None, None, :].to(x.dtype)) * -10000.0).to(x.dtype)
        mask_i32 = None if dense else attention_mask.to(torch.int32).contiguous()
        for layer in self.layers:
            x = layer(x, bias, mask_i32)
        return _qa_head(x, self.qa)


def init_weights(model, seed=0):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) * 0.02)
                if isinstance(m, nn.Linear) and m.bias is not None:
                    m.bias.zero_()
            elif isinstance(m, nn.LayerNorm):
                m.weight.fill_(1.0)
                m.bias.zero_()


# GEMM solutions measured on MI355X for the bert_large bucket shapes (every
# projection at batch 1..64 x seq 384) by PyTorch TunableOp over hipBLASLt and
# rocBLAS (tools/bert_probe.py --tunable); see use_tuned_gemms.
TUNED_GEMMS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "bert_large_gfx950.csv")


def use_tuned_gemms(path=TUNED_GEMMS):
    """Route torch's GEMMs through TunableOp with the measured solution table
    (tuning itself stays off: a shape missing from the table runs the
    library's default solution).  The table's validators (PyTorch, HIP,
    hipBLASLt, rocBLAS, gfx arch) must match this process, else TunableOp stays
    off.  Off by default: TunableOp is process-wide (every torch GEMM of every
    model in the server process would go through it) and the table measured
    neutral within noise in served runs (profiles/r4_bench_bert_tunable_on.json
    vs _off.json).  TC_BERT_TUNED_GEMMS=1 turns it on (bert-only server
    processes).  Returns True when it is on."""
    if os.environ.get("TC_BERT_TUNED_GEMMS", "0") != "1" or not os.path.exists(path) or not torch.cuda.is_available():
        return False
    import torch.cuda.tunable as tun

    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    tun.enable(True)
    if not tun.read_file(path):
        tun.enable(False)
        return False
    return True


def build(device="cuda", dtype=torch.bfloat16, seed=0, layers=LAYERS):
    model = BertLargeQA(layers)
    init_weights(model, seed)
    return model.eval().to(device=device, dtype=dtype)


def flops_per_sequence(seq=384, layers=LAYERS):
    """Forward FLOPs of one sequence (GEMMs + attention), for reporting."""
    gemm = 2 * seq * (HIDDEN * 3 * HIDDEN + HIDDEN * HIDDEN + 2 * HIDDEN * FFN)
    attn = 2 * 2 * seq * seq * HIDDEN
    return layers * (gemm + attn) + 2 * seq * HIDDEN * 2


def _check_head_dim():
    assert HIDDEN % HEADS == 0 and math.log2(HIDDEN // HEADS).is_integer()
