"""PDNN_TUNE key checking across the two halves of the dispatch table: the kernel library reports the keys its
table (csrc/kernels/tuning.h) does not have and the Python side accepts those of ITS table (tuning.py), so
neither keeps a copy of the other's key list; a key in neither table makes the library fail to load."""
import os
import re
import subprocess
import sys
from pathlib import Path

from pytorch_distributed_nn_amd import tuning

ROOT = Path(__file__).resolve().parent.parent


def _load_with(tune):
    code = "from pytorch_distributed_nn_amd.ops import _backend; print(_backend.available(), _backend._ERR)"
    env = dict(os.environ, PDNN_TUNE=tune, PYTHONPATH=str(ROOT))
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120).stdout


def test_python_and_kernel_keys_accepted_unknown_rejected():
    py = next(iter(tuning.DEFAULTS))
    out = _load_with(f"{py}={tuning.DEFAULTS[py]},glds=1")
    assert out.startswith("True"), out
    out = _load_with("no_such_key=1")
    assert out.startswith("False") and "no_such_key" in out, out


def test_docstring_documents_every_python_key():
    for k in tuning.DEFAULTS:
        assert re.search(rf"^{k}\s+{tuning.DEFAULTS[k]}\s", tuning.__doc__, re.M), k
