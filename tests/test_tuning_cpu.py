"""The kernel library accepts the Python-side dispatch-table keys in PDNN_TUNE (csrc/kernels/tuning.hip keeps
their list): the two must not drift apart."""
import re
from pathlib import Path

from pytorch_distributed_nn_amd import tuning


def test_kernel_library_knows_every_python_key():
    src = (Path(__file__).resolve().parent.parent / "csrc" / "kernels" / "tuning.hip").read_text()
    m = re.search(r"keys\[\]\s*=\s*\{([^}]*)\}", src)
    assert m, "python-key list not found in tuning.hip"
    keys = set(re.findall(r'"(\w+)"', m.group(1)))
    assert keys == set(tuning.DEFAULTS)


def test_docstring_documents_every_python_key():
    for k in tuning.DEFAULTS:
        assert re.search(rf"^{k}\s+{tuning.DEFAULTS[k]}\s", tuning.__doc__, re.M), k
