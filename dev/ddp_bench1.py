"""bench.py on ONE GPU through the DDP/RCCL path (1-rank nccl group, communication forced on), without a
launcher process, so it can run directly under rocprofv3: python tools/ddp_bench1.py [bench args]."""
import os
import runpy
import sys

os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                  MASTER_PORT=os.environ.get("MASTER_PORT", "29613"), PDNN_FORCE_PG="1", PDNN_DDP_FORCE_COMM="1")
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.argv = [os.path.join(root, "bench.py"), "--steps", "3", "--warmup", "3", *sys.argv[1:]]
runpy.run_path(sys.argv[0], run_name="__main__")
