"""fp32-parity DenseNet-121 inference engine on the split-precision CDNA4
kernels K8x-K10x (csrc/kernels/densenet_x3.hip).

This is the engine behind the headline ``densenet_onnx`` number: the
reference's model contract is FP32 (reference
src/python/examples/image_client.py:84-86 sends FP32 tensors to an fp32 ONNX
graph), so the served logits must match an fp32 DenseNet-121, not a bf16 one.
Every conv runs as a "bf16x3" product on the bf16 MFMA
(a*b ~= a_hi*b_hi + a_hi*b_lo + a_lo*b_hi, fp32 accumulate): ~1e-5 relative
per conv, at 3/16 of the cost of gfx950's f32-input MFMA.

Network walk (same as :class:`densenet_fused.FusedDenseNet`, fp32 activations):

  per-image fp32 NCHW device pointers (the server's request regions, never
  assembled into a batch)
   -> K10x stem: relu(maxpool(conv0 7x7/2) + b0)        -> block-1 buffer ch[0:64]
   -> per dense layer:  K8x conv1x1 (BN1+ReLU prologue; BN2-folded bias+ReLU
                        epilogue) -> z as split bf16 planes [pixels,128] x 2
                        K9x conv3x3 z -> block buffer ch[c_in : c_in+32] (fp32)
                        (one x3_dense_layer call; small-M layers run the 1x1
                        split-K and the 3x3 reduces its partials in-kernel)
                        or (K <= 224, 16 <= W <= 56; K <= 480 at >= 4 tiles
                        per block): K11x, the whole layer in ONE kernel with z
                        produced into the 3x3's LDS ring (never in HBM)
                        or, small M (<= 3136 pixels, W <= 63): the K13x chain,
                        one launch per layer (csrc/kernels/densenet_x3s.hip)
                        or (14x14 / 7x7 blocks from ~16-32 images): K14x, one
                        launch per layer over row tiles of the images (2-4
                        per image, halo rows recomputed), z in a zero-padded
                        LDS image of the tile
   -> per transition:   K8x conv1x1 with BN+ReLU+2x2 avg-pool prologue
                        -> next block buffer ch[0 : C/2] (fp32)
   -> K10x head: relu(BN5(x)) global average -> [b,1024] fp32
   -> classifier: fp32 GEMM (hipBLASLt) -> fp32 logits

All launches go to the caller's current HIP stream with no host sync, so a
forward captures into one HIP graph per batch bucket.
"""

import os

import torch
import torch.nn.functional as F

from triton_client_amd.ops import hip

from .densenet import BLOCKS, BN_SIZE, GROWTH, INIT_FEATURES  # noqa: F401
from .densenet_fused import _bn_affine

IMG_ELEMS = 3 * 224 * 224
FUSE_MAX_K = 224  # K11x at every batch: K 64..224
FUSE_MAX_K_BIG = 480  # ... and up to K 480 (the late block-2 layers) from fuse_big_k_min_tiles tiles per block


def split_bf16(w):
    """fp32 tensor -> (hi, lo) bf16 tensors with w ~= hi + lo (RNE both)."""
    w = w.float()
    hi = w.to(torch.bfloat16)
    lo = (w - hi.float()).to(torch.bfloat16)
    return hi.contiguous(), lo.contiguous()


class FusedDenseNetFP32:
    """Split weights + per-batch-capacity fp32 activation buffers."""

    H0 = 224
    precision = "fp32"

    def __init__(self, model, max_batch, device):
        assert all(layer.folded for blk in model.blocks for layer in blk), "call fold_for_inference first"
        dev = torch.device(device)
        self.device = dev
        with torch.no_grad():
            s0, b0 = _bn_affine(model.norm0)
            w0 = model.conv0.weight.float() * s0.view(-1, 1, 1, 1)
            # K10x layout: [64][kh 7][kw 8][ch 4], zero at kw 7 / ch 3
            w0p = torch.zeros(w0.shape[0], 7, 8, 4)
            w0p[:, :, :7, :3] = w0.permute(0, 2, 3, 1).cpu()
            self.w0_hi, self.w0_lo = (hip.x3_stem_fragments(t).to(dev)
                                      for t in split_bf16(w0p.reshape(w0.shape[0], -1)))
            self.b0 = b0.to(dev).contiguous()
            self.blocks, self.trans, self.block_dims = [], [], []
            hw, c = self.H0 // 4, INIT_FEATURES
            for bi, layers in enumerate(model.blocks):
                ctot = c + len(layers) * GROWTH
                ls = []
                for j, layer in enumerate(layers):
                    cin = c + j * GROWTH
                    s1, t1 = _bn_affine(layer.norm1)
                    w1h, w1l = split_bf16(layer.conv1.weight.reshape(BN_SIZE * GROWTH, cin))
                    # [32][128][3][3] -> [32][3][3][128] (tap-major K)
                    w2h, w2l = split_bf16(layer.conv2.weight.permute(0, 2, 3, 1).reshape(GROWTH, -1))
                    ls.append({
                        "cin": cin, "s1": s1.to(dev), "t1": t1.to(dev),
                        "w1h": w1h.to(dev), "w1l": w1l.to(dev),
                        "b1": layer.conv1.bias.float().to(dev).contiguous(),
                        "w2h": hip.x3_w3_fragments(w2h).to(dev), "w2l": hip.x3_w3_fragments(w2l).to(dev),
                        # K11x (fused layer) fragment layouts
                        "w1fh": hip.x3_w1_fragments(w1h).to(dev), "w1fl": hip.x3_w1_fragments(w1l).to(dev),
                        "w2fh": hip.x3_w3f_fragments(w2h).to(dev), "w2fl": hip.x3_w3f_fragments(w2l).to(dev),
                    })
                self.blocks.append(ls)
                self.block_dims.append((hw, ctot))
                c = ctot
                if bi < len(model.transitions):
                    t = model.transitions[bi]
                    st, tt = _bn_affine(t.norm)
                    wh, wl = split_bf16(t.conv.weight.reshape(c // 2, c))
                    self.trans.append({"s": st.to(dev), "t": tt.to(dev), "wh": wh.to(dev), "wl": wl.to(dev)})
                    c //= 2
                    hw //= 2
            s5, t5 = _bn_affine(model.norm5)
            self.s5, self.t5 = s5.to(dev), t5.to(dev)
            self.wc = model.classifier.weight.float().to(dev).contiguous()
            self.bc = model.classifier.bias.float().to(dev).contiguous()
            self.num_features = c
        # K11x runs a layer when every block gets at least this many 64-pixel
        # tiles (its per-block prologue recomputes a (2W+2)-row halo of z, yet it
        # still beats the two-launch pair at bs1); 0 disables it (A/B runs)
        self.fuse_min_tiles = int(os.environ.get("TCAMD_X3_FUSE_MIN_TPB", "1"))
        # ... and past K = 224 from this many tiles per block: 1 (K11x for K 256..480
        # at any batch: engine bs12-48 +1..6 % against the pair there, round 5;
        # from bs64 every block has >= 4 tiles anyway; profiles/r5_engine_ab.md)
        self.fuse_big_k_min_tiles = int(os.environ.get("TCAMD_X3_FUSE_BIGK_MIN_TPB", "1"))
        # K11x v3 (the next chunk's 1x1 interleaved into the 3x3) on blocks of
        # width >= fuse_v3 at >= 2 tiles per block; 0 = v1 everywhere.  Engine
        # bs128 x 2 streams 47.1k -> 47.6k img/s with v3 on both K11x blocks
        # (profiles/r5_k11x_v3.md)
        self.fuse_v3 = int(os.environ.get("TCAMD_X3_FUSE_V3", "28"))
        # ... from this many 64-pixel tiles per CU (engine attribute)
        self.fuse_v3_tiles_per_cu = 2
        # K13x (small-M dense layer, csrc/kernels/densenet_x3s.hip) for the
        # unfused layers of a block with at most this many pixels; 0 disables it
        self.small_m = int(os.environ.get("TCAMD_X3_SMALL_M", "1600"))
        # ... and, up to chain_m pixels (W <= 63), the K13x chain (one launch per
        # layer); TCAMD_X3_CHAIN=0: two launches per layer up to small_m
        self.use_chain = os.environ.get("TCAMD_X3_CHAIN", "1") != "0"
        self.chain_m = int(os.environ.get("TCAMD_X3_CHAIN_M", "3136"))
        # K14x (whole dense layer in one kernel at 14x14 / 7x7) once the launch
        # has at least this many workgroups (images x row tiles: 2-4 per 14x14
        # image, 1-4 per 7x7 image, x3_small_tiles); 0 disables it.  Unset:
        # 48 when the engine is one of several concurrent streams (a server's
        # model instances: concurrent_streams), else 64 -- K14x beats the
        # K13x chain from bs12 on two streams (+6 / +13 / +19 % at bs12 / 14 /
        # 16) but only from bs20 on one (profiles/r5_engine_ab.md)
        env = os.environ.get("TCAMD_X3_SMALLF_MIN_BLOCKS")
        self.smallf_min_blocks = int(env) if env else None
        self.concurrent_streams = 1
        # tiles per image for K14x: 0 = the library's chip-filling choice
        self.smallf_tiles = int(os.environ.get("TCAMD_X3_SMALLF_TILES", "0"))
        self._alloc(max_batch)

    def _alloc(self, n):
        """fp32 activation buffers for up to ``n`` images (one set per concurrent stream)."""
        dev = self.device
        self.max_batch = int(n)
        self.feat = [torch.empty(n * hw * hw, ct, device=dev, dtype=torch.float32) for hw, ct in self.block_dims]
        h1 = self.block_dims[0][0]
        self.z_hi = torch.empty(n * h1 * h1, BN_SIZE * GROWTH, device=dev, dtype=torch.bfloat16)
        self.z_lo = torch.empty_like(self.z_hi)
        self.pooled = torch.empty(n, self.num_features, device=dev, dtype=torch.float32)
        self.ptrs = torch.zeros(n, device=dev, dtype=torch.int64)
        self._img_off = torch.arange(n, device=dev, dtype=torch.int64) * (IMG_ELEMS * 4)
        # split-K partials: the largest request over every 1x1 conv at EVERY
        # batch size up to n (small batches split the most; sized for n alone,
        # a capacity-256 serving engine found no room and ran bs1 unsplit)
        need = 0
        for bi, layers in enumerate(self.blocks):
            hw, ctot = self.block_dims[bi]
            for cin in sorted({L["cin"] for L in layers}):
                need = max(need, max(hip.x3_conv1x1_ws_bytes(b * hw * hw, cin) for b in range(1, n + 1)))
            if bi < len(self.trans):
                nhw = self.block_dims[bi + 1][0]
                need = max(need, max(hip.x3_conv1x1_ws_bytes(b * nhw * nhw, ctot, ctot // 2)
                                     for b in range(1, n + 1)))
        self.ws = torch.empty(max(need, 16), device=dev, dtype=torch.uint8)
        # K13x ping-pong 1x1 accumulators: a layer adds into one (zero on
        # entry) and its 3x3 zeroes the other for the next layer
        rows = max([b * hw * hw for hw, _ in self.block_dims for b in range(1, n + 1)
                    if b * hw * hw <= self.small_m] or [0])
        self.zacc = torch.zeros(2, max(rows, 1), BN_SIZE * GROWTH, device=dev, dtype=torch.float32)
        # K13x chain (one launch per small-M layer, W <= 63): a zacc per layer of
        # every block that can run it, and a device table of layer entries
        self.chain = []
        for bi, layers in enumerate(self.blocks):
            hw = self.block_dims[bi][0]
            rows = max([b * hw * hw for b in range(1, n + 1) if b * hw * hw <= self.chain_m] or [0])
            if not self.use_chain or rows == 0 or hw > 63:
                self.chain.append(None)
                continue
            zc = torch.empty(len(layers), rows, BN_SIZE * GROWTH, device=dev, dtype=torch.float32)
            ent = [hip.x3c_layer_entry(L["w1fh"].data_ptr(), L["w1fl"].data_ptr(), L["s1"].data_ptr(),
                                       L["t1"].data_ptr(), L["b1"].data_ptr(), L["w2h"].data_ptr(),
                                       L["w2l"].data_ptr(), zc[j].data_ptr(), L["cin"]) for j, L in enumerate(layers)]
            table = torch.tensor(ent, dtype=torch.int64).to(dev)
            self.chain.append((zc, table, rows))

    def with_workspace(self, max_batch=None):
        """A second engine sharing these weights with its own activation buffers."""
        import copy

        other = copy.copy(self)
        other._alloc(self.max_batch if max_batch is None else max_batch)
        return other

    def forward(self, x, out=None):
        """x: [b,3,224,224] fp32 NCHW contiguous; returns/fills [b,1000] fp32."""
        b = int(x.shape[0])
        if b > self.max_batch:
            raise ValueError("batch %d exceeds capacity %d" % (b, self.max_batch))
        if x.dtype != torch.float32 or not x.is_contiguous() or tuple(x.shape[1:]) != (3, self.H0, self.H0):
            x = x.float().contiguous()
        self.ptrs[:b] = self._img_off[:b] + x.data_ptr()
        self._x_keepalive = x
        return self.forward_ptrs(b, out)

    def forward_ptrs(self, b, out=None):
        """Run ``b`` images whose fp32 NCHW [3,224,224] device pointers are in ``self.ptrs[:b]``."""
        if b > self.max_batch:
            raise ValueError("batch %d exceeds capacity %d" % (b, self.max_batch))
        st = torch.cuda.current_stream(self.device).cuda_stream
        hw0, c0 = self.block_dims[0]
        hip.x3_stem(self.ptrs.data_ptr(), self.w0_hi.data_ptr(), self.w0_lo.data_ptr(), self.b0.data_ptr(),
                    self.feat[0].data_ptr(), b, c0, stream=st)
        ws, wsb = self.ws.data_ptr(), self.ws.numel()
        zh, zl = self.z_hi.data_ptr(), self.z_lo.data_ptr()
        zacc = None  # K13x: index of the zeroed accumulator, None before the first small layer
        for bi, layers in enumerate(self.blocks):
            hw, ctot = self.block_dims[bi]
            fp = self.feat[bi].data_ptr()
            M = b * hw * hw
            fused = self._fuse(M, hw)
            fmax = self._fuse_max_k(M)
            small = 0 < M <= self.small_m and M <= self.zacc.shape[1]
            if self._small_fused(b, hw):
                # K14x: the 14x14 / 7x7 blocks, one launch per layer, z on chip
                for L in layers:
                    hip.x3_dense_small(fp, ctot, b, hw, hw, L["cin"], L["s1"].data_ptr(), L["t1"].data_ptr(),
                                       L["w1fh"].data_ptr(), L["w1fl"].data_ptr(), L["b1"].data_ptr(),
                                       L["w2fh"].data_ptr(), L["w2fl"].data_ptr(), fp + 4 * L["cin"], ctot, stream=st,
                                       tiles=self._small_tiles(b, hw))
                self._transition(bi, fp, ctot, b, hw, ws, wsb, st)
                continue
            ch = self.chain[bi]
            if ch is not None and 0 < M <= ch[2]:
                # the whole block runs as one chain (at bs1-2 a 28x28 K11x layer
                # takes 13-15 us, a chain layer ~5.5; starting the chain after
                # the layers K11x would take lost, round 3)
                tab, n = ch[1].data_ptr(), len(layers)
                hip.x3c_base(tab, n, fp, ctot, b, hw, hw, stream=st)
                for i in range(n):
                    hip.x3c_layer(tab, i, n, fp, ctot, b, hw, hw, stream=st)
                self._transition(bi, fp, ctot, b, hw, ws, wsb, st)
                continue
            for L in layers:
                if fused and L["cin"] <= fmax:
                    self._fused_layer(fused, L, fp, ctot, b, hw, st)
                    continue
                if small:
                    # M only shrinks from here on, so the rows each 3x3 zeroes
                    # cover every later layer's
                    if zacc is None:
                        zacc = 0
                        self.zacc[0, :M].zero_()
                    hip.x3s_dense_layer(fp, ctot, b, hw, hw, L["cin"], L["s1"].data_ptr(), L["t1"].data_ptr(),
                                        L["w1fh"].data_ptr(), L["w1fl"].data_ptr(), L["b1"].data_ptr(),
                                        self.zacc[zacc].data_ptr(), self.zacc[zacc ^ 1].data_ptr(),
                                        L["w2h"].data_ptr(), L["w2l"].data_ptr(), fp + 4 * L["cin"], ctot, stream=st)
                    zacc ^= 1
                    continue
                hip.x3_dense_layer(fp, ctot, b, hw, hw, L["cin"], L["s1"].data_ptr(), L["t1"].data_ptr(),
                                   L["w1h"].data_ptr(), L["w1l"].data_ptr(), L["b1"].data_ptr(), zh, zl,
                                   L["w2h"].data_ptr(), L["w2l"].data_ptr(), fp + 4 * L["cin"], ctot, ws=ws,
                                   ws_bytes=wsb, stream=st)
            self._transition(bi, fp, ctot, b, hw, ws, wsb, st)
        hw4, c4 = self.block_dims[-1]
        hip.x3_head_pool(self.feat[-1].data_ptr(), self.s5.data_ptr(), self.t5.data_ptr(), self.pooled.data_ptr(),
                         b, hw4 * hw4, c4, stream=st)
        if out is None:
            return F.linear(self.pooled[:b], self.wc, self.bc)
        torch.addmm(self.bc, self.pooled[:b], self.wc.t(), out=out[:b])
        return out[:b]

    __call__ = forward

    def _fused_layer(self, fused, L, fp, ctot, b, hw, st):
        """K11x: the whole dense layer in one kernel.  v3 (the next chunk's 1x1
        interleaved into each tile's 3x3) on blocks of width >= fuse_v3 once every
        block walks >= 2 tiles; v1 elsewhere (bs1 included: one tile per block
        has no next chunk to interleave).  The 4-wave v2 of rounds 3-4 lost in
        the whole forward and was removed (profiles/r5_k11x_v3.md)."""
        args = (fp, ctot, b, hw, hw, L["cin"], L["s1"].data_ptr(), L["t1"].data_ptr(), L["w1fh"].data_ptr(),
                L["w1fl"].data_ptr(), L["b1"].data_ptr(), L["w2fh"].data_ptr(), L["w2fl"].data_ptr(),
                fp + 4 * L["cin"], ctot)
        if self.fuse_v3 and hw >= self.fuse_v3 and b * hw * hw >= self.fuse_v3_tiles_per_cu * 64 * _cu_count(self.device):
            hip.x3_dense_fused3(*args, stream=st)
        else:
            hip.x3_dense_fused(*args, stream=st)

    def _transition(self, bi, fp, ctot, b, hw, ws, wsb, st):
        if bi < len(self.trans):
            T = self.trans[bi]
            nhw, nct = self.block_dims[bi + 1]
            hip.x3_conv1x1(fp, ctot, b * nhw * nhw, ctot, T["s"].data_ptr(), T["t"].data_ptr(),
                           T["wh"].data_ptr(), T["wl"].data_ptr(), y=self.feat[bi + 1].data_ptr(), ldy=nct,
                           pool=1, H=hw, W=hw, ws=ws, ws_bytes=wsb, stream=st, N=ctot // 2)

    def _small_tiles(self, b, hw):
        """K14x row tiles per image: TCAMD_X3_SMALLF_TILES, else the native
        chip-filling choice, except that the 7-tile split of small 14x14 batches
        must fit one round of this stream's share of the CUs (on 2 streams at
        bs32 it oversubscribes them: -5.6 %, profiles/r5_k14x_tiles.md)."""
        if self.smallf_tiles:
            return self.smallf_tiles
        return stream_share_tiles(hip.x3_small_tiles(b, hw), b, _cu_count(self.device), self.concurrent_streams)

    def _small_fused(self, b, hw):
        thr = self.smallf_min_blocks
        if thr is None:
            # one stream: from 16 images (with 7-tile 14x14 layers K14x is 7 % faster
            # there, 2 % slower at 12; profiles/r5_k14x_tiles.md)
            thr = 48 if self.concurrent_streams > 1 else 64
        if thr <= 0 or hw not in (7, 14):
            return False
        # the thresholds count workgroups at up to 4 row tiles per image (the
        # 7-tile split of small 14x14 batches came later and did not move them)
        tiles = min(self._small_tiles(b, hw), 4)
        return b * tiles >= thr

    def _fuse_max_k(self, M):
        """Largest K that K11x takes: past 224 only at >= 4 tiles per block, where
        v1 beats the pair by 8-15% per layer at 28x28 (K 256..480, bs128; at bs32
        it loses at K >= 384: profiles/r3_fused_dense_layer.md)."""
        tiles = (M + 63) // 64
        per_block = -(-tiles // min(tiles, _cu_count(self.device)))
        return FUSE_MAX_K_BIG if per_block >= self.fuse_big_k_min_tiles else FUSE_MAX_K

    def _fuse(self, M, W):
        """K11x (whole layer, z in LDS) for this block's layers: 0 = no (K8x + K9x
        pair), otherwise yes (1 / 2: small / big batch)."""
        if self.fuse_min_tiles <= 0 or W > 56 or W < 16:
            return 0
        tiles = (M + 63) // 64
        per_block = -(-tiles // min(tiles, _cu_count(self.device)))
        if per_block < self.fuse_min_tiles:
            return 0
        return 2 if (W >= 56 and per_block >= 4) else 1


_CU = {}


def stream_share_tiles(native_tiles, imgs, ncu, streams):
    """K14x tiles per image given the native chip-filling choice: its 7-tile
    split of small 14x14 batches only while the grid fits one round of this
    stream's share of the CUs, else quarters."""
    if native_tiles == 7 and (imgs + 7) // 8 * 8 * 7 > ncu // max(1, streams):
        return 4
    return native_tiles


def _cu_count(dev):
    key = str(dev)
    if key not in _CU:
        _CU[key] = torch.cuda.get_device_properties(dev).multi_processor_count
    return _CU[key]


def build(max_batch, device="cuda", seed=0):
    """Random-init, BN-calibrated, folded DenseNet-121 as an fp32-parity engine.
    Returns (engine, the fp32 torch module it must match)."""
    from . import densenet

    model = densenet.DenseNet121()
    densenet.init_weights(model, seed)
    densenet.calibrate_bn(model, device="cpu")
    densenet.fold_for_inference(model)
    model.eval()
    return FusedDenseNetFP32(model, max_batch, device), model
