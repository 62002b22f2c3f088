"""pytorch_distributed_nn_amd — an MI355X-native distributed data-parallel training framework.

Same capabilities as chao1224/pytorch_distributed_nn (parameter-server sync SGD with k-of-n straggler
kill / backup workers / short-circuit, bucketed all-reduce DDP, LeNet/ResNet/MLP model zoo, native
C++ MLP trainer), re-designed for AMD Instinct MI355X: one process per GPU over RCCL/xGMI,
hand-written HIP/CDNA4 kernels for the hot ops, fused flat-buffer optimizers.
"""
__version__ = "0.1.0"
