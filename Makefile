# Native build + run targets (reference MPI_code/Makefile:1-19).
#   make                  kernels (hipcc, gfx950) + host runtime + the pdnn_mlp CLI
#   make single_run       CPP-11: single-machine native MLP
#   make distributed_run  CPP-01: master + evaluator + (NP-2) workers over the TCP store, NP=8
#   make test             CPU test-suite
PY ?= python3
NP ?= 8
ITERS ?= 50
COLLECT ?= 2
BIN = pytorch_distributed_nn_amd/_lib/pdnn_mlp

all: kernels runtime $(BIN)

kernels:
	$(PY) -m pytorch_distributed_nn_amd._build kernels

runtime:
	$(PY) -m pytorch_distributed_nn_amd._build runtime

$(BIN): csrc/tools/pdnn_mlp.cpp csrc/runtime/*.cpp csrc/runtime/runtime.h
	$(PY) -m pytorch_distributed_nn_amd._build tools

single_run: $(BIN)
	$(BIN) single --iters $(ITERS)

distributed_run: $(BIN)
	mkdir -p outfiles && $(BIN) distributed --nprocs $(NP) --collect $(COLLECT) --iters $(ITERS) --out outfiles/

test:
	$(PY) -m pytest tests/ -x -q -m "not gpu"

.PHONY: all kernels runtime single_run distributed_run test
