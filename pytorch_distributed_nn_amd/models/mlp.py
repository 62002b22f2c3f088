"""Fully-connected model zoo of the reference stacks.

* ``mlp2``           — BASELINE.json config 1: 2-layer MLP on MNIST-shaped tensors (784 -> 512 -> 10, ReLU).
* ``mlp_cpp``        — the native C++ PS MLP (MPI_code/src/distributed_nn.cpp:35-47):
                       784-500-500-800-800-200-100-100-10, sigmoid hidden units, softmax output.
* ``mlp_s2``         — the NumPy PS MLP (pure_py_code/distributed_nn.py:41-96): 28 FC layers
                       784-500-500-800x22-200-100-10 with sigmoid.
* ``mlp_tf``         — the TF ``fc_inference`` model (distributed_TF/src/mnist.py:150-412): 29 dense
                       sigmoid layers 784-500-500-800x23-200-200-100-10.
* :class:`TFConvNet` — the TF ``inference`` conv net (distributed_TF/src/mnist.py:77-148):
                       conv5x5x32-pool-conv5x5x64-pool-fc512-dropout-fc10 (SAME padding).

Hidden layers are ``nn.Linear`` modules named ``fc{i}`` so checkpoints are plain state_dicts; on the GPU
each Linear is one MFMA GEMM with the bias (and a ReLU) fused in the epilogue, sigmoid is a vectorised
elementwise kernel.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import functional as OF


class MLP(nn.Module):
    def __init__(self, sizes, activation="relu", init_std=None):
        super().__init__()
        self.sizes = list(sizes)
        self.activation = activation
        for i in range(len(sizes) - 1):
            lin = nn.Linear(sizes[i], sizes[i + 1])
            if init_std is not None:   # the reference NumPy/C++ stacks use Gaussian init (nn_layer.h:235-239)
                nn.init.normal_(lin.weight, 0.0, init_std)
                nn.init.zeros_(lin.bias)
            setattr(self, f"fc{i}", lin)
        self.n_layers = len(sizes) - 1

    def forward(self, x):
        x = x.reshape(x.shape[0], -1)
        gpu = x.is_cuda
        for i in range(self.n_layers):
            lin = getattr(self, f"fc{i}")
            last = i == self.n_layers - 1
            if gpu:
                x = OF.linear(x, lin.weight, lin.bias, relu=(not last and self.activation == "relu"))
                if not last and self.activation == "sigmoid":
                    x = OF.sigmoid(x)
            else:
                x = F.linear(x, lin.weight, lin.bias)
                if not last:
                    x = F.relu(x) if self.activation == "relu" else torch.sigmoid(x)
        return x


def mlp2(num_classes=10, hidden=512):
    return MLP([784, hidden, num_classes], "relu")


def mlp_cpp(num_classes=10):
    return MLP([784, 500, 500, 800, 800, 200, 100, 100, num_classes], "sigmoid")


def mlp_s2(num_classes=10):
    return MLP([784, 500, 500] + [800] * 23 + [200, 100, num_classes], "sigmoid")


def mlp_tf(num_classes=10):
    return MLP([784, 500, 500] + [800] * 23 + [200, 200, 100, num_classes], "sigmoid")


class TFConvNet(nn.Module):
    def __init__(self, num_classes=10, in_channels=1, dropout=0.5):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, 32, 5, 1, 2)
        self.conv2 = nn.Conv2d(32, 64, 5, 1, 2)
        self.fc1 = nn.Linear(7 * 7 * 64, 512)
        self.fc2 = nn.Linear(512, num_classes)
        self.dropout = dropout

    def forward(self, x):
        if x.is_cuda:
            h = OF.nchw_to_nhwc_input(x)
            h = OF.max_pool2d_nhwc(OF.relu(OF.conv2d_nhwc(h, self.conv1.weight, 1, 2, self.conv1.bias)), 2, 2)
            h = OF.max_pool2d_nhwc(OF.relu(OF.conv2d_nhwc(h, self.conv2.weight, 1, 2, self.conv2.bias)), 2, 2)
            h = h.permute(0, 3, 1, 2).reshape(h.shape[0], -1)
            h = OF.linear(h, self.fc1.weight, self.fc1.bias, relu=True)
            if self.training and self.dropout:
                h = F.dropout(h, self.dropout)
            return OF.linear(h, self.fc2.weight, self.fc2.bias)
        h = F.max_pool2d(F.relu(self.conv1(x)), 2)
        h = F.max_pool2d(F.relu(self.conv2(h)), 2)
        h = F.relu(self.fc1(h.flatten(1)))
        h = F.dropout(h, self.dropout, self.training)
        return self.fc2(h)
