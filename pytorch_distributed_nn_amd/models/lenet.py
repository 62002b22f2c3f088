"""LeNet (reference: pytorch_code/model_ops/lenet.py:12-33).

conv5x5(1->20) -> maxpool2 -> relu -> conv5x5(20->50) -> maxpool2 -> relu -> fc(800->500) -> fc(500->10).
Note the reference has NO activation between fc1 and fc2 (lenet.py:28-29); we keep that exactly, and the
parameter names conv1/conv2/fc1/fc2 so reference state_dicts load unchanged.

The reference's ``LeNetSplit`` (lenet.py:35-225) detaches every layer boundary so it can push each
gradient to the parameter server as soon as it exists; here that early-push behaviour is provided by
the DDP bucket hooks / PS gradient streaming (``parallel/``), so one model class serves both.

GPU path: NHWC bf16 through the HIP conv / pool / GEMM kernels; channel counts 1/20/50 are padded to
multiples of 8 on the fly (padding channels stay exactly zero) and the flatten uses the reference's
NCHW order so ``fc1.weight`` means the same thing on both paths.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import functional as OF


class LeNet(nn.Module):
    fused = True

    def __init__(self, num_classes=10):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 20, 5, 1)
        self.conv2 = nn.Conv2d(20, 50, 5, 1)
        self.fc1 = nn.Linear(4 * 4 * 50, 500)
        self.fc2 = nn.Linear(500, num_classes)

    def forward(self, x):
        if x.is_cuda and self.fused:
            return self.forward_nhwc(x)
        x = F.relu(F.max_pool2d(self.conv1(x), 2, 2))
        x = F.relu(F.max_pool2d(self.conv2(x), 2, 2))
        x = x.reshape(-1, 4 * 4 * 50)
        return self.fc2(self.fc1(x))

    def forward_nhwc(self, x):
        h = OF.nchw_to_nhwc_input(x)                              # [N,28,28,8]
        h = OF.conv2d_nhwc(h, self.conv1.weight, 1, 0, self.conv1.bias)   # [N,24,24,24]
        h = OF.relu(OF.max_pool2d_nhwc(h, 2, 2))
        h = OF.conv2d_nhwc(h, self.conv2.weight, 1, 0, self.conv2.bias)   # [N,8,8,56]
        h = OF.relu(OF.max_pool2d_nhwc(h, 2, 2))                   # [N,4,4,56]
        h = h[..., :50].permute(0, 3, 1, 2).reshape(h.shape[0], -1)   # reference NCHW flatten order
        h = OF.linear(h, self.fc1.weight, self.fc1.bias)
        return OF.linear(h, self.fc2.weight, self.fc2.bias)

    def name(self):
        return "lenet"
