"""ResNet family.

* :class:`ResNet` — the reference's CIFAR-stem ResNet (pytorch_code/model_ops/resnet.py:67-113):
  3x3 stem, stages 64/128/256/512, ``avg_pool2d(4)``, ``linear`` head, ``shortcut`` downsample.
  state_dict keys are identical to the reference (``conv1.weight``, ``layer2.0.shortcut.0.weight``,
  ``linear.weight`` ...), so reference checkpoints load unchanged.
* :class:`ResNetImageNet` — the standard 224x224 ImageNet ResNet (7x7/2 stem + 3x3/2 max-pool,
  stride on the 3x3 conv of the bottleneck, ``fc`` head, torchvision key names incl. ``downsample``).
  This is the headline benchmark model (BASELINE.json: ResNet-50 DDP samples/sec).

GPU path: the network runs on NHWC bf16 activations through the block-level fused HIP ops of
``ops.fused_resnet`` (one autograd node per block).  CPU path: the reference forward on NCHW fp32
torch ops — used by the CPU test-suite and as the numerics reference of the GPU path.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import functional as OF
from ..ops import kernels as K
from ..ops.fused_resnet import BasicBlockFn, BottleneckFn, StemFn, side_forward, stem_shadow


def _bn_conf(bn: nn.BatchNorm2d):
    mom = bn.momentum if bn.momentum is not None else 0.1
    return mom, bn.eps


class _FusedBlockMixin:
    expansion = 1
    ds_name = "shortcut"

    def _ds(self):
        d = getattr(self, self.ds_name)
        return d if len(d) else None

    def _block_params(self):
        convs, bns = self._convs_bns()
        ds = self._ds()
        if ds is not None:
            convs.append(ds[0])
            bns.append(ds[1])
        params, bufs, shadows = [], [], []
        for c, b in zip(convs, bns):
            params += [c.weight, b.weight, b.bias]
            bufs += [b.running_mean, b.running_var]
            shadows.append(OF.weight_bf16(c.weight, krsc=True))
        return params, bufs, shadows, bns


class BasicBlock(_FusedBlockMixin, nn.Module):
    expansion = 1

    def __init__(self, in_planes, planes, stride=1, ds_name="shortcut"):
        super().__init__()
        self.ds_name = ds_name
        self.stride = stride
        self.conv1 = nn.Conv2d(in_planes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        ds = nn.Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            ds = nn.Sequential(nn.Conv2d(in_planes, self.expansion * planes, 1, stride, bias=False),
                               nn.BatchNorm2d(self.expansion * planes))
        setattr(self, ds_name, ds)

    def _convs_bns(self):
        return [self.conv1, self.conv2], [self.bn1, self.bn2]

    def forward(self, x):          # reference semantics (resnet.py:31-36), NCHW
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        out = out + getattr(self, self.ds_name)(x)
        return F.relu(out)

    def forward_nhwc(self, x):     # fused GPU path
        params, bufs, shadows, bns = self._block_params()
        mom, eps = _bn_conf(self.bn1)
        return BasicBlockFn.apply(x, (self.stride, self.training, mom, eps), bufs, shadows, *params)


class Bottleneck(_FusedBlockMixin, nn.Module):
    expansion = 4

    def __init__(self, in_planes, planes, stride=1, ds_name="shortcut"):
        super().__init__()
        self.ds_name = ds_name
        self.stride = stride
        self.conv1 = nn.Conv2d(in_planes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, self.expansion * planes, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(self.expansion * planes)
        ds = nn.Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            ds = nn.Sequential(nn.Conv2d(in_planes, self.expansion * planes, 1, stride, bias=False),
                               nn.BatchNorm2d(self.expansion * planes))
        setattr(self, ds_name, ds)

    def _convs_bns(self):
        return [self.conv1, self.conv2, self.conv3], [self.bn1, self.bn2, self.bn3]

    def forward(self, x):          # reference semantics (resnet.py:58-64), NCHW
        out = F.relu(self.bn1(self.conv1(x)))
        out = F.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        out = out + getattr(self, self.ds_name)(x)
        return F.relu(out)

    fp8 = False                    # conv2 (3x3, stride 1) forward + data gradient on the fp8 halo kernel (enable_fp8)

    def forward_nhwc(self, x):
        params, bufs, shadows, bns = self._block_params()
        mom, eps = _bn_conf(self.bn1)
        meta = None
        if self.fp8 and self.stride == 1 and self.conv2.out_channels % 128 == 0:
            meta = getattr(self, "_fp8_state", None)
            if meta is None:
                from ..ops.fused_resnet import Fp8Conv2
                meta = self._fp8_state = Fp8Conv2(x.device)
        return BottleneckFn.apply(x, (self.stride, self.training, mom, eps, meta), bufs, shadows, *params)


class _ResNetBase(nn.Module):
    fused = True   # GPU tensors run the fused HIP path

    def awaits_params(self, x, *args, **kwargs):
        """Whether this forward fetches every conv / linear weight through await_param itself (the fused GPU path:
        bf16 shadows): then DistributedDataParallel's k-of-n forward needs no per-op ParamUseMode dispatch."""
        return bool(getattr(x, "is_cuda", False) and self.fused)

    def _bn_modules(self):
        if not hasattr(self, "_bn_cache"):
            self._bn_cache = [m for m in self.modules() if isinstance(m, nn.BatchNorm2d)]
        return self._bn_cache

    def _count_bn_batches(self):
        if self.training:
            t = [m.num_batches_tracked for m in self._bn_modules() if m.num_batches_tracked is not None]
            if t:
                torch._foreach_add_(t, 1)

    def _blocks(self):
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            yield from layer

    def _prefetch_fp8(self, x):
        """fp8 mode: the 3x3 convs' e4m3 weights made on the side stream while the stem runs."""
        if not x.is_cuda:
            return
        ps = [b.conv2.weight for b in self._blocks() if getattr(b, "fp8", False) and b.stride == 1
              and b.conv2.out_channels % 128 == 0]
        if not ps:
            return
        from ..ops.fused_resnet import _side_stream
        side = _side_stream(x.device)
        if side is not None:
            from ..ops.fp8 import prefetch_fp8_weights
            prefetch_fp8_weights(ps, side)


class ResNet(_ResNetBase):
    """CIFAR-stem ResNet, exactly the reference architecture and parameter names."""

    def __init__(self, block, num_blocks, num_classes=10):
        super().__init__()
        self.in_planes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.layer1 = self._make_layer(block, 64, num_blocks[0], 1)
        self.layer2 = self._make_layer(block, 128, num_blocks[1], 2)
        self.layer3 = self._make_layer(block, 256, num_blocks[2], 2)
        self.layer4 = self._make_layer(block, 512, num_blocks[3], 2)
        self.linear = nn.Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, n, stride):
        layers = []
        for s in [stride] + [1] * (n - 1):
            layers.append(block(self.in_planes, planes, s, "shortcut"))
            self.in_planes = planes * block.expansion
        return nn.Sequential(*layers)

    def forward(self, x):
        if x.is_cuda and self.fused:
            return self.forward_nhwc(x)
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.layer4(self.layer3(self.layer2(self.layer1(out))))
        out = F.avg_pool2d(out, 4)
        return self.linear(out.reshape(out.size(0), -1))

    def enable_fp8(self, on: bool = True):
        """BASELINE.json config 5: the bottlenecks' stride-1 3x3 convs run their forward (e4m3 activations) and data
        gradient (e5m2 gradients) on the fp8 halo kernel (block-scaled MFMA, per-tensor delayed scaling, the operand
        quantised in-line); weight gradients and the 1x1 convs stay bf16."""
        for m in self.modules():
            if isinstance(m, Bottleneck):
                m.fp8 = on
        return self

    def forward_nhwc(self, x):
        xin = OF.nchw_to_nhwc_input(x)
        mom, eps = _bn_conf(self.bn1)
        self._count_bn_batches()
        out = StemFn.apply(xin, (1, 1, False, self.training, mom, eps), [self.bn1.running_mean, self.bn1.running_var],
                           [stem_shadow(self.conv1.weight, xin.shape[-1])], self.conv1.weight, self.bn1.weight,
                           self.bn1.bias)
        for b in self._blocks():
            out = b.forward_nhwc(out)
        out = OF.avg_pool2d_nhwc(out, 4)
        return OF.linear(out.reshape(out.shape[0], -1), self.linear.weight, self.linear.bias)


class ResNetImageNet(_ResNetBase):
    """224x224 ImageNet ResNet (torchvision layout / key names)."""

    def __init__(self, block, layers, num_classes=1000, zero_init_residual=False):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0], 1)
        self.layer2 = self._make_layer(block, 128, layers[1], 2)
        self.layer3 = self._make_layer(block, 256, layers[2], 2)
        self.layer4 = self._make_layer(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make_layer(self, block, planes, n, stride):
        layers = []
        for s in [stride] + [1] * (n - 1):
            layers.append(block(self.inplanes, planes, s, "downsample"))
            self.inplanes = planes * block.expansion
        return nn.Sequential(*layers)

    def forward(self, x):
        if x.is_cuda and self.fused:
            return self.forward_nhwc(x)
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))

    def enable_fp8(self, on: bool = True):
        """BASELINE.json config 5: the bottlenecks' stride-1 3x3 convs run their forward (e4m3 activations) and data
        gradient (e5m2 gradients) on the fp8 halo kernel (block-scaled MFMA, per-tensor delayed scaling, the operand
        quantised in-line); weight gradients and the 1x1 convs stay bf16."""
        for m in self.modules():
            if isinstance(m, Bottleneck):
                m.fp8 = on
        return self

    def forward_nhwc(self, x):
        mom, eps = _bn_conf(self.bn1)
        self._count_bn_batches()
        conf = (2, 3, True, self.training, mom, eps)
        bufs = [self.bn1.running_mean, self.bn1.running_var]
        params = (self.conv1.weight, self.bn1.weight, self.bn1.bias)
        self._prefetch_fp8(x)            # on the side stream, beside the stem
        if K.stem_nchw_ok(x):
            # the stem kernel reads the NCHW batch directly (csrc/kernels/stem.hip stem7n_kernel)
            xb = x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16)
            out = StemFn.apply(xb.contiguous(), conf, bufs, [K.stem_weight_nchw(self.conv1.weight)], *params)
        else:
            xin = OF.nchw_to_nhwc_input(x)
            out = StemFn.apply(xin, conf, bufs, [stem_shadow(self.conv1.weight, xin.shape[-1])], *params)
        with side_forward(out.device):
            for b in self._blocks():
                out = b.forward_nhwc(out)
        feat = OF.global_avg_pool_nhwc(out)
        return OF.linear(feat, self.fc.weight, self.fc.bias)


# ---- factories (reference: resnet.py:100-113) ---------------------------------------------------------
def ResNet18(num_classes=10):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes)


def ResNet34(num_classes=10):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes)


def ResNet50(num_classes=10):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes)


def ResNet101(num_classes=10):
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes)


def ResNet152(num_classes=10):
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes)


def resnet18_imagenet(num_classes=1000):
    return ResNetImageNet(BasicBlock, [2, 2, 2, 2], num_classes)


def resnet34_imagenet(num_classes=1000):
    return ResNetImageNet(BasicBlock, [3, 4, 6, 3], num_classes)


def resnet50_imagenet(num_classes=1000):
    return ResNetImageNet(Bottleneck, [3, 4, 6, 3], num_classes)


def resnet101_imagenet(num_classes=1000):
    return ResNetImageNet(Bottleneck, [3, 4, 23, 3], num_classes)


def resnet152_imagenet(num_classes=1000):
    return ResNetImageNet(Bottleneck, [3, 8, 36, 3], num_classes)
