"""Build the kernel library of another git revision next to the current one, for same-box A/B runs
(``PDNN_KERNEL_LIB=<path> python bench.py`` loads it instead of the in-tree build).

python dev/probes/build_base.py REV OUT.so"""
import os
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    rev, out = sys.argv[1], Path(sys.argv[2]).resolve()
    from pytorch_distributed_nn_amd import _build as B
    root = B.ROOT
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        arch = subprocess.run(["git", "-C", str(root), "archive", rev, "csrc"], check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", str(td)], input=arch, check=True)
        flags = [f for f in B.HIP_FLAGS if not f.startswith("-I")]
        flags += [f"-I{td / 'csrc' / 'include'}", f"-I{td / 'csrc' / 'kernels'}"]
        srcs = sorted((td / "csrc" / "kernels").glob("*.hip"))
        deps = sorted((td / "csrc" / "kernels").glob("*.h")) + sorted((td / "csrc" / "include").glob("*.h"))
        out.parent.mkdir(parents=True, exist_ok=True)
        B._build_lib(srcs, B.HIPCC, flags, out, td / "obj", deps, file_flags=B.KERNEL_FILE_FLAGS)
    print(out)


if __name__ == "__main__":
    main()
