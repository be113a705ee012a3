"""DenseNet-121 for the ``densenet_onnx`` bench model (random-init weights).

Architecture follows the public DenseNet-121 (growth 32, blocks 6/12/24/16,
bn_size 4, 224x224 input, 1000 classes) that Triton's ``densenet_onnx``
example model implements; there is no ONNX runtime or checkpoint on the box,
so weights are random (seeded) and BatchNorm statistics are calibrated once
on a random batch so activations stay well-scaled through all 121 layers.

Inference-time rewrites (exact up to floating-point rounding):

* BN that FOLLOWS a conv (norm2 after conv1 in every dense layer) is folded
  into that conv's weight/bias;
* transition layers apply the 2x2 average pool BEFORE their 1x1 conv (both
  are linear and commute), a 4x FLOP/byte cut for those convs;
* everything runs channels_last (NHWC) in bf16 — the layout MIOpen's
  MFMA-based convolutions want on CDNA4 — with fp32 logits out.

The serving wrapper (server/gpu_models.py) captures one HIP graph per batch
bucket so a forward costs one graph launch instead of ~400 kernel launches.
"""

import torch
import torch.nn as nn
import torch.nn.functional as F

BLOCKS = (6, 12, 24, 16)
GROWTH = 32
BN_SIZE = 4
INIT_FEATURES = 64
NUM_CLASSES = 1000


class _DenseLayer(nn.Module):
    def __init__(self, cin):
        super().__init__()
        self.norm1 = nn.BatchNorm2d(cin)
        self.conv1 = nn.Conv2d(cin, BN_SIZE * GROWTH, 1, bias=False)
        self.norm2 = nn.BatchNorm2d(BN_SIZE * GROWTH)
        self.conv2 = nn.Conv2d(BN_SIZE * GROWTH, GROWTH, 3, padding=1, bias=False)
        self.folded = False

    def forward(self, x):
        y = self.conv1(F.relu(self.norm1(x)))
        if not self.folded:
            y = self.norm2(y)
        return self.conv2(F.relu(y))


class _Transition(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.norm = nn.BatchNorm2d(cin)
        self.conv = nn.Conv2d(cin, cout, 1, bias=False)
        self.pool_first = False

    def forward(self, x):
        x = F.relu(self.norm(x))
        if self.pool_first:
            return self.conv(F.avg_pool2d(x, 2, 2))
        return F.avg_pool2d(self.conv(x), 2, 2)


class DenseNet121(nn.Module):
    def __init__(self, num_classes=NUM_CLASSES):
        super().__init__()
        self.conv0 = nn.Conv2d(3, INIT_FEATURES, 7, stride=2, padding=3, bias=False)
        self.norm0 = nn.BatchNorm2d(INIT_FEATURES)
        blocks = []
        trans = []
        c = INIT_FEATURES
        for i, n in enumerate(BLOCKS):
            layers = nn.ModuleList()
            for j in range(n):
                layers.append(_DenseLayer(c + j * GROWTH))
            blocks.append(layers)
            c = c + n * GROWTH
            if i != len(BLOCKS) - 1:
                trans.append(_Transition(c, c // 2))
                c = c // 2
        self.blocks = nn.ModuleList(blocks)
        self.transitions = nn.ModuleList(trans)
        self.norm5 = nn.BatchNorm2d(c)
        self.classifier = nn.Linear(c, num_classes)
        self.num_features = c

    def forward(self, x):
        x = F.relu(self.norm0(self.conv0(x)))
        x = F.max_pool2d(x, 3, 2, 1)
        for i, layers in enumerate(self.blocks):
            feats = [x]
            for layer in layers:
                feats.append(layer(torch.cat(feats, 1) if len(feats) > 1 else feats[0]))
            x = torch.cat(feats, 1)
            if i < len(self.transitions):
                x = self.transitions[i](x)
        x = F.relu(self.norm5(x))
        x = F.adaptive_avg_pool2d(x, 1).flatten(1)
        return self.classifier(x)


def init_weights(model, seed=0):
    g = torch.Generator().manual_seed(seed)
    for m in model.modules():
        if isinstance(m, nn.Conv2d):
            fan_in = m.in_channels * m.kernel_size[0] * m.kernel_size[1]
            m.weight.data = torch.randn(m.weight.shape, generator=g) * (2.0 / fan_in) ** 0.5
        elif isinstance(m, nn.BatchNorm2d):
            m.weight.data = 1.0 + 0.1 * torch.randn(m.weight.shape, generator=g)
            m.bias.data = 0.05 * torch.randn(m.bias.shape, generator=g)
            m.running_mean.zero_()
            m.running_var.fill_(1.0)
        elif isinstance(m, nn.Linear):
            m.weight.data = torch.randn(m.weight.shape, generator=g) * (1.0 / m.in_features) ** 0.5
            m.bias.data.zero_()


@torch.no_grad()
def calibrate_bn(model, batch=8, seed=1, device="cpu"):
    """Set BN running stats from one random batch (momentum 1)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(batch, 3, 224, 224, generator=g).to(device)
    moms = {}
    for m in model.modules():
        if isinstance(m, nn.BatchNorm2d):
            moms[m] = m.momentum
            m.momentum = 1.0
    model.train()
    model(x)
    model.eval()
    for m, mom in moms.items():
        m.momentum = mom


@torch.no_grad()
def fold_for_inference(model):
    """Apply the exact inference rewrites (BN-after-conv fold, pool-first)."""
    for layers in model.blocks:
        for layer in layers:
            if layer.folded:
                continue
            bn = layer.norm2
            scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
            w = layer.conv1.weight * scale.view(-1, 1, 1, 1)
            b = bn.bias - bn.running_mean * scale
            conv = nn.Conv2d(layer.conv1.in_channels, layer.conv1.out_channels, 1, bias=True)
            conv.weight.data = w
            conv.bias.data = b
            layer.conv1 = conv.to(w.device)
            layer.folded = True
    for t in model.transitions:
        t.pool_first = True
    return model


def build(device="cuda", dtype=torch.bfloat16, seed=0, fold=True):
    """Random-init, BN-calibrated, inference-folded DenseNet-121."""
    model = DenseNet121()
    init_weights(model, seed)
    calibrate_bn(model, device="cpu")
    if fold:
        fold_for_inference(model)
    model = model.eval().to(device=device, dtype=dtype)
    model = model.to(memory_format=torch.channels_last)
    return model
