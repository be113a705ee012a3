"""DenseNet-121 inference engine on the hand-written CDNA4 kernels (K8-K10).

Executes the same network as :class:`densenet.DenseNet121` (after
``fold_for_inference``) without per-op library calls:

  x [b,224,224,3] bf16 NHWC, or a device table of per-image fp32 NCHW
  pointers (``forward_ptrs``: the server's requests, never assembled)
   -> K10s  relu(maxpool(conv0 7x7/2) + b0)      -> block-1 buffer ch[0:64]
            (one kernel: BN0 folded into the conv weight, conv tile in LDS;
            ``stem="miopen"`` keeps the library conv + K10a for comparison)
   -> per dense layer:   K8 conv1x1 (BN1+ReLU prologue, BN2-folded bias+ReLU
                         epilogue) -> z [pixels,128]
                         K9 conv3x3 z -> block buffer ch[c_in : c_in+32]
   -> per transition:    K8 conv1x1 with BN+ReLU+2x2 avg-pool prologue
                         -> next block buffer ch[0 : C/2]
   -> K10b  relu(BN5(x)) global average -> [b,1024] bf16
   -> classifier (hipBLASLt linear) -> fp32 logits

All feature maps of a dense block live in ONE preallocated NHWC buffer
(channels = block input + 32 * layers), so DenseNet's concatenations cost
nothing.  Every launch goes to the caller's current HIP stream and no host
synchronisation happens inside ``forward``, so the whole forward captures
into a single HIP graph per batch bucket (server/gpu_models.py).
"""

import torch
import torch.nn.functional as F

from triton_client_amd.ops import hip

from .densenet import BLOCKS, GROWTH, BN_SIZE, INIT_FEATURES


def _bn_affine(bn):
    scale = (bn.weight.float() / torch.sqrt(bn.running_var.float() + bn.eps))
    bias = bn.bias.float() - bn.running_mean.float() * scale
    return scale.contiguous(), bias.contiguous()


class FusedDenseNet:
    """Weights re-laid-out for K8/K9 + per-batch-capacity activation buffers."""

    H0 = 224

    def __init__(self, model, max_batch, device, stem="fused"):
        assert all(layer.folded for blk in model.blocks for layer in blk), "call fold_for_inference first"
        dev = torch.device(device)
        bf = torch.bfloat16
        self.device = dev
        self.max_batch = int(max_batch)
        if stem not in ("fused", "miopen"):
            raise ValueError("stem must be 'fused' or 'miopen'")
        self.stem = stem
        with torch.no_grad():
            s0, b0 = _bn_affine(model.norm0)
            w0 = model.conv0.weight.float() * s0.view(-1, 1, 1, 1)
            self.w0 = w0.to(dev, bf).contiguous(memory_format=torch.channels_last)
            # K10s layout: [64][kh 7][kw 8][ch 4], zero at kw 7 / ch 3
            w0p = torch.zeros(w0.shape[0], 7, 8, 4)
            w0p[:, :, :7, :3] = w0.permute(0, 2, 3, 1).cpu()
            self.w0p = w0p.reshape(w0.shape[0], -1).to(dev, bf).contiguous()
            self.b0 = b0.to(dev)
            self.blocks = []
            self.trans = []
            hw = self.H0 // 4
            c = INIT_FEATURES
            self.block_dims = []
            for bi, layers in enumerate(model.blocks):
                ctot = c + len(layers) * GROWTH
                ls = []
                for j, layer in enumerate(layers):
                    cin = c + j * GROWTH
                    s1, t1 = _bn_affine(layer.norm1)
                    w1 = layer.conv1.weight.reshape(BN_SIZE * GROWTH, cin)
                    ls.append({
                        "cin": cin,
                        "s1": s1.to(dev), "t1": t1.to(dev),
                        "w1": w1.to(dev, bf).contiguous(),
                        "b1": layer.conv1.bias.float().to(dev).contiguous(),
                        # [32][128][3][3] -> [32][3][3][128] (tap-major K for the implicit GEMM)
                        "w2": layer.conv2.weight.permute(0, 2, 3, 1).to(dev, bf).contiguous(),
                    })
                self.blocks.append(ls)
                self.block_dims.append((hw, ctot))
                c = ctot
                if bi < len(model.transitions):
                    t = model.transitions[bi]
                    st, tt = _bn_affine(t.norm)
                    self.trans.append({
                        "s": st.to(dev), "t": tt.to(dev),
                        "w": t.conv.weight.reshape(c // 2, c).to(dev, bf).contiguous(),
                    })
                    c //= 2
                    hw //= 2
            s5, t5 = _bn_affine(model.norm5)
            self.s5, self.t5 = s5.to(dev), t5.to(dev)
            self.wc = model.classifier.weight.to(dev, bf).contiguous()
            self.bc = model.classifier.bias.to(dev, bf).contiguous()
            self.num_features = c
        self._alloc(self.max_batch)

    def _alloc(self, n):
        """Activation buffers for up to ``n`` images (one set per concurrent stream)."""
        dev, bf = self.device, torch.bfloat16
        self.max_batch = int(n)
        self.feat = [torch.empty(n * hw_ * hw_, ct, device=dev, dtype=bf) for hw_, ct in self.block_dims]
        h1 = self.block_dims[0][0]
        self.z = torch.empty(n * h1 * h1, BN_SIZE * GROWTH, device=dev, dtype=bf)
        self.pooled = torch.empty(n, self.num_features, device=dev, dtype=bf)
        # per-image fp32 NCHW input pointers read by K10s (forward_ptrs)
        self.ptrs = torch.zeros(n, device=dev, dtype=torch.int64)
        # split-K fp32 partials for the small-M 1x1 convs (K8 splits only while
        # its grid is < 128 blocks, so splits * M * N <= 16 * 128 * 32 * 128)
        self.ws = torch.empty(16 * 128 * 32 * 128 * 4, device=dev, dtype=torch.uint8)

    def with_workspace(self, max_batch=None):
        """A second engine sharing these weights with its own activation buffers,
        so model instances on different HIP streams can run concurrently."""
        import copy

        other = copy.copy(self)
        other._alloc(self.max_batch if max_batch is None else max_batch)
        return other

    def forward(self, x, out=None):
        """x: [b,3,224,224] bf16 channels_last (NHWC memory); returns/fills [b,1000] fp32."""
        b = int(x.shape[0])
        if b > self.max_batch:
            raise ValueError("batch %d exceeds capacity %d" % (b, self.max_batch))
        st = torch.cuda.current_stream(self.device).cuda_stream
        if self.stem == "fused":
            if x.dtype != torch.bfloat16 or not x.is_contiguous(memory_format=torch.channels_last):
                x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            hip.dn_stem_fused(None, x.data_ptr(), self.w0p.data_ptr(), self.b0.data_ptr(), self.feat[0].data_ptr(),
                              b, self.block_dims[0][1], stream=st)
        else:
            self._stem_miopen(x, b, st)
        return self._trunk(b, st, out)

    def forward_ptrs(self, b, out=None):
        """Run ``b`` images whose fp32 NCHW [3,224,224] device pointers are in ``self.ptrs[:b]``."""
        if b > self.max_batch:
            raise ValueError("batch %d exceeds capacity %d" % (b, self.max_batch))
        st = torch.cuda.current_stream(self.device).cuda_stream
        hip.dn_stem_fused(self.ptrs.data_ptr(), None, self.w0p.data_ptr(), self.b0.data_ptr(),
                          self.feat[0].data_ptr(), b, self.block_dims[0][1], stream=st)
        return self._trunk(b, st, out)

    def _stem_miopen(self, x, b, st):
        y0 = F.conv2d(x, self.w0, stride=2, padding=3)  # [b,64,112,112] channels_last
        if not y0.is_contiguous(memory_format=torch.channels_last):
            y0 = y0.contiguous(memory_format=torch.channels_last)
        h0 = int(y0.shape[2])
        hip.dn_stem_pool(y0.data_ptr(), self.b0.data_ptr(), self.feat[0].data_ptr(), b, h0, h0, INIT_FEATURES,
                         self.block_dims[0][1], stream=st)

    def _trunk(self, b, st, out):
        for bi, layers in enumerate(self.blocks):
            hw, ctot = self.block_dims[bi]
            feat = self.feat[bi]
            fp = feat.data_ptr()
            M = b * hw * hw
            for L in layers:
                hip.dn_conv1x1(fp, ctot, M, L["cin"], L["s1"].data_ptr(), L["t1"].data_ptr(), L["w1"].data_ptr(),
                               BN_SIZE * GROWTH, L["b1"].data_ptr(), 1, self.z.data_ptr(), BN_SIZE * GROWTH,
                               stream=st, ws=self.ws.data_ptr(), ws_bytes=self.ws.numel())
                hip.dn_conv3x3(self.z.data_ptr(), b, hw, hw, L["w2"].data_ptr(), fp + 2 * L["cin"], ctot, stream=st)
            if bi < len(self.trans):
                T = self.trans[bi]
                nhw, nct = self.block_dims[bi + 1]
                hip.dn_conv1x1(fp, ctot, b * nhw * nhw, ctot, T["s"].data_ptr(), T["t"].data_ptr(),
                               T["w"].data_ptr(), ctot // 2, None, 0, self.feat[bi + 1].data_ptr(), nct,
                               pool=1, H=hw, W=hw, stream=st, ws=self.ws.data_ptr(), ws_bytes=self.ws.numel())
        hw4, c4 = self.block_dims[-1]
        hip.dn_head_pool(self.feat[-1].data_ptr(), self.s5.data_ptr(), self.t5.data_ptr(), self.pooled.data_ptr(),
                         b, hw4 * hw4, c4, stream=st)
        logits = F.linear(self.pooled[:b], self.wc, self.bc)
        if out is None:
            return logits.float()
        out[:b].copy_(logits)
        return out[:b]

    __call__ = forward


def build(max_batch, device="cuda", seed=0, stem="fused"):
    """Random-init, BN-calibrated, folded DenseNet-121 as a fused engine."""
    from . import densenet

    model = densenet.DenseNet121()
    densenet.init_weights(model, seed)
    densenet.calibrate_bn(model, device="cpu")
    densenet.fold_for_inference(model)
    model.eval()
    return FusedDenseNet(model, max_batch, device, stem=stem), model
