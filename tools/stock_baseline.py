"""Stock PyTorch-ROCm comparison line ("run stock PyTorch-ROCm DDP on the same box").

Builds a torchvision-equivalent ResNet-50 (ImageNet stem, 224x224, 1000 classes) out of plain
``torch.nn`` modules (torchvision is not installed here), trains it with synthetic data and reports
samples/sec.  This is the number the framework's own ``bench.py`` has to beat; it uses MIOpen for
conv/BN and hipBLASLt for the FC layer.

    python tools/stock_baseline.py --batch 256 --steps 20 --warmup 5 [--mode bf16|autocast|fp32]
"""
import argparse
import json
import os
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inp, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(inp, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.down = None
        if stride != 1 or inp != planes * 4:
            self.down = nn.Sequential(nn.Conv2d(inp, planes * 4, 1, stride, bias=False),
                                      nn.BatchNorm2d(planes * 4))

    def forward(self, x):
        o = F.relu(self.bn1(self.conv1(x)))
        o = F.relu(self.bn2(self.conv2(o)))
        o = self.bn3(self.conv3(o))
        return F.relu(o + (x if self.down is None else self.down(x)))


class ResNet50(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        inp, blocks = 64, []
        for i, (n, planes) in enumerate(zip(layers, (64, 128, 256, 512))):
            for j in range(n):
                blocks.append(Bottleneck(inp, planes, 2 if (j == 0 and i > 0) else 1))
                inp = planes * 4
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.bn1(self.conv1(x))), 3, 2, 1)
        x = self.blocks(x)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", default="bf16", choices=["bf16", "autocast", "fp32"])
    ap.add_argument("--channels-last", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    torch.cuda.set_device(dev)
    torch.backends.cudnn.benchmark = True
    m = ResNet50().to(dev)
    mf = torch.channels_last if a.channels_last else torch.contiguous_format
    if a.mode == "bf16":
        m = m.to(torch.bfloat16)
    m = m.to(memory_format=mf)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    xdt = torch.bfloat16 if a.mode == "bf16" else torch.float32
    x = torch.randn(a.batch, 3, 224, 224, device=dev, dtype=xdt).to(memory_format=mf)
    y = torch.randint(0, 1000, (a.batch,), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(a.mode == "autocast")):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": "stock_resnet50_samples_per_sec", "mode": a.mode, "batch": a.batch,
                      "channels_last": a.channels_last, "value": a.batch * a.steps / dt,
                      "ms_per_step": 1e3 * dt / a.steps, "loss": float(loss)}), flush=True)


if __name__ == "__main__":
    main()
