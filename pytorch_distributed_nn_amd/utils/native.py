"""ctypes bindings of the C++ host runtime ``_lib/libpdnn_runtime.so`` (csrc/runtime/).

* :class:`StoreServer` / :class:`Store` — control-plane TCP key/value store (step epochs, kill flags,
  heartbeats, evaluator run name, metrics side-channel).
* :class:`PSCoordinator` — parameter-server gradient-collection state machine (full sync, k-of-n kill,
  backup workers with stale-by-step drop, arrival timeline).
* :func:`idx_read` / :func:`idx_write` — MNIST IDX files.
* :class:`NativeMLP` and :func:`run_native_role` — the native MLP trainer and its master / worker /
  evaluator roles (the C++/MPI stack of the reference, MPI_code/, re-hosted on the store).
"""
from __future__ import annotations

import ctypes
import os
import struct
from pathlib import Path

import numpy as np

_LIB = None
_P, _I, _L, _F, _D, _U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_double, ctypes.c_uint64
_CP = ctypes.c_char_p

_SIGS = {
    "pdnn_store_server_start": (_P, [_I]),
    "pdnn_store_server_port": (_I, [_P]),
    "pdnn_store_server_stop": (None, [_P]),
    "pdnn_store_connect": (_P, [_CP, _I, _I]),
    "pdnn_store_close": (None, [_P]),
    "pdnn_store_set": (_I, [_P, _CP, _P, _U64]),
    "pdnn_store_get": (_I, [_P, _CP, _L]),
    "pdnn_store_wait": (_I, [_P, _CP, _L]),
    "pdnn_store_add": (_L, [_P, _CP, _L]),
    "pdnn_store_push": (_L, [_P, _CP, _P, _U64]),
    "pdnn_store_check": (_I, [_P, _CP]),
    "pdnn_store_del": (_I, [_P, _CP]),
    "pdnn_store_keys": (_I, [_P, _CP]),
    "pdnn_store_last_len": (_U64, [_P]),
    "pdnn_store_copy_last": (None, [_P, _P]),
    "pdnn_ps_create": (_P, [_I, _I, _I, _I]),
    "pdnn_ps_destroy": (None, [_P]),
    "pdnn_ps_begin_step": (None, [_P, _L]),
    "pdnn_ps_offer": (_I, [_P, _I, _I, _L, _D]),
    "pdnn_ps_done": (_I, [_P]),
    "pdnn_ps_close": (None, [_P]),
    "pdnn_ps_count": (_I, [_P, _I]),
    "pdnn_ps_stragglers": (_I, [_P, _I, _P]),
    "pdnn_ps_contributed": (_I, [_P, _I, _I]),
    "pdnn_ps_stale_dropped": (_L, [_P]),
    "pdnn_ps_timeline": (_I, [_P, _P, _P, _P, _P, _I]),
    "pdnn_idx_read": (_I, [_CP, _P, _L, _P, _P]),
    "pdnn_idx_write": (_I, [_CP, _P, _P, _I, _I]),
    "pdnn_shuffle_indices": (None, [_P, _L, _U64]),
    "pdnn_mlp_create": (_P, [_P, _I, _I, _F, _U64]),
    "pdnn_mlp_destroy": (None, [_P]),
    "pdnn_mlp_n_layers": (_I, [_P]),
    "pdnn_mlp_layer_size": (_L, [_P, _I]),
    "pdnn_mlp_weights": (ctypes.POINTER(ctypes.c_float), [_P, _I]),
    "pdnn_mlp_grads": (ctypes.POINTER(ctypes.c_float), [_P, _I]),
    "pdnn_mlp_forward_backward": (_F, [_P, _P, _P, _I]),
    "pdnn_mlp_apply": (None, [_P, _F]),
    "pdnn_mlp_loss": (_F, [_P, _P, _P, _I, _P]),
    "pdnn_mlp_train_single": (_I, [_P, _P, _P, _I, _I, _P]),
    "pdnn_mlp_run_role": (_I, [_CP, _CP, _I, _I, _I, _I, _I, _P, _P, _I, _P, _I, _I, _F, _I, _CP]),
}


def lib():
    global _LIB
    if _LIB is None:
        p = Path(__file__).resolve().parent.parent / "_lib" / "libpdnn_runtime.so"
        from .. import _build
        if not p.exists():
            _build.build_runtime()          # under an inter-process lock; objects renamed into place
        elif _build.stale_sources("runtime"):
            import warnings
            warnings.warn(f"{p} is older than its C++ sources; rebuild with `python -m pytorch_distributed_nn_amd._build`")
        l = ctypes.CDLL(str(p))
        for n, (res, args) in _SIGS.items():
            f = getattr(l, n)
            f.restype = res
            f.argtypes = args
        _LIB = l
    return _LIB


def _np_ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------------------------------- store
class StoreServer:
    def __init__(self, port: int = 0):
        self.h = lib().pdnn_store_server_start(port)
        if not self.h:
            raise OSError(f"could not start control-plane store on port {port}")
        self.port = lib().pdnn_store_server_port(self.h)

    def stop(self):
        if self.h:
            lib().pdnn_store_server_stop(self.h)
            self.h = None

    def __del__(self):
        try:
            self.stop()
        except Exception:
            pass


class StoreTimeout(TimeoutError):
    pass


class Store:
    """Client of the control-plane store.  Values are bytes; helpers for int64 and str."""

    def __init__(self, host: str = "127.0.0.1", port: int = 29600, timeout_ms: int = 30000):
        self.h = lib().pdnn_store_connect(host.encode(), port, timeout_ms)
        if not self.h:
            raise ConnectionError(f"cannot connect to store {host}:{port}")

    def close(self):
        if self.h:
            lib().pdnn_store_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _last(self) -> bytes:
        n = lib().pdnn_store_last_len(self.h)
        buf = ctypes.create_string_buffer(n)
        lib().pdnn_store_copy_last(self.h, buf)
        return buf.raw[:n]

    def set(self, key: str, value) -> None:
        if isinstance(value, str):
            value = value.encode()
        if isinstance(value, np.ndarray):
            value = value.tobytes()
        b = bytes(value)
        buf = ctypes.create_string_buffer(b, len(b))
        if lib().pdnn_store_set(self.h, key.encode(), buf, len(b)) != 0:
            raise ConnectionError("store set failed")

    def get(self, key: str, timeout_ms: int = -1) -> bytes:
        st = lib().pdnn_store_get(self.h, key.encode(), timeout_ms)
        if st == 1:
            raise StoreTimeout(key)
        if st != 0:
            raise ConnectionError(f"store get {key} failed ({st})")
        return self._last()

    def wait(self, key: str, timeout_ms: int = -1) -> bool:
        return lib().pdnn_store_wait(self.h, key.encode(), timeout_ms) == 0

    def add(self, key: str, delta: int = 1) -> int:
        return lib().pdnn_store_add(self.h, key.encode(), delta)

    def push(self, queue: str, value) -> int:
        """Append to a queue in one round trip: n = ++``<queue>_n``, ``<queue>/<n>`` = value; returns n."""
        b = value.encode() if isinstance(value, str) else bytes(value)
        buf = ctypes.create_string_buffer(b, len(b))
        n = lib().pdnn_store_push(self.h, queue.encode(), buf, len(b))
        if n == -2 ** 63:
            raise ConnectionError("store push failed")
        return n

    def check(self, key: str) -> bool:
        return lib().pdnn_store_check(self.h, key.encode()) == 1

    def delete(self, key: str) -> None:
        lib().pdnn_store_del(self.h, key.encode())

    def keys(self, prefix: str = "") -> list[str]:
        lib().pdnn_store_keys(self.h, prefix.encode())
        return [k for k in self._last().decode().split("\n") if k]

    def set_int(self, key: str, v: int):
        self.set(key, struct.pack("<q", v))

    def get_int(self, key: str, timeout_ms: int = -1) -> int:
        return struct.unpack("<q", self.get(key, timeout_ms))[0]


# ---------------------------------------------------------------------------------------- PS state machine
class PSCoordinator:
    ACCEPTED, STALE, DUPLICATE, CLOSED, BAD, FUTURE = range(6)

    def __init__(self, n_workers: int, n_layers: int, n_to_collect: int = 0, kill_k: int = 0):
        self.n_workers, self.n_layers = n_workers, n_layers
        self.h = lib().pdnn_ps_create(n_workers, n_layers, n_to_collect, kill_k)

    def __del__(self):
        try:
            lib().pdnn_ps_destroy(self.h)
        except Exception:
            pass

    def begin_step(self, step: int):
        lib().pdnn_ps_begin_step(self.h, step)

    def offer(self, worker: int, layer: int, step: int, t_ms: float = 0.0) -> int:
        return lib().pdnn_ps_offer(self.h, worker, layer, step, t_ms)

    def done(self) -> bool:
        return bool(lib().pdnn_ps_done(self.h))

    def close(self):
        """Close the step regardless of counts (interval / deadline): later offers are rejected."""
        lib().pdnn_ps_close(self.h)

    def count(self, layer: int) -> int:
        return lib().pdnn_ps_count(self.h, layer)

    def stragglers(self, sentinel_layer: int = 0) -> list[int]:
        out = (ctypes.c_int * self.n_workers)()
        n = lib().pdnn_ps_stragglers(self.h, sentinel_layer, out)
        return list(out[:n])

    def contributed(self, layer: int, worker: int) -> bool:
        return bool(lib().pdnn_ps_contributed(self.h, layer, worker))

    @property
    def stale_dropped(self) -> int:
        return lib().pdnn_ps_stale_dropped(self.h)

    def timeline(self):
        cap = 1 << 16
        t = np.zeros(cap, np.float64)
        s = np.zeros(cap, np.int64)
        w = np.zeros(cap, np.int32)
        l = np.zeros(cap, np.int32)
        n = min(cap, lib().pdnn_ps_timeline(self.h, _np_ptr(t), _np_ptr(s), _np_ptr(w), _np_ptr(l), cap))
        return list(zip(t[:n].tolist(), s[:n].tolist(), w[:n].tolist(), l[:n].tolist()))


# ---------------------------------------------------------------------------------------- IDX
def idx_read(path) -> np.ndarray:
    dims = (ctypes.c_int * 4)()
    nd = ctypes.c_int()
    rc = lib().pdnn_idx_read(str(path).encode(), None, 0, dims, ctypes.byref(nd))
    if rc not in (-4,):
        raise ValueError(f"bad IDX file {path} ({rc})")
    shape = tuple(dims[: nd.value])
    out = np.empty(shape, np.uint8)
    rc = lib().pdnn_idx_read(str(path).encode(), _np_ptr(out), out.size, dims, ctypes.byref(nd))
    if rc != out.size:
        raise ValueError(f"truncated IDX file {path} ({rc})")
    return out


def idx_write(path, arr: np.ndarray) -> None:
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    dims = (ctypes.c_int * arr.ndim)(*arr.shape)
    if lib().pdnn_idx_write(str(path).encode(), _np_ptr(arr), dims, arr.ndim, 0x08) != 0:
        raise OSError(f"cannot write {path}")


def shuffle_indices(n: int, seed: int) -> np.ndarray:
    idx = np.arange(n, dtype=np.int64)
    lib().pdnn_shuffle_indices(_np_ptr(idx), n, seed)
    return idx


# ---------------------------------------------------------------------------------------- native MLP
class NativeMLP:
    """C++ MLP with bias-folded weights (the reference's MPI_code NN/NNLayer)."""

    def __init__(self, sizes, batch=128, lr=1e-3, seed=1234):
        self.sizes = np.asarray(sizes, np.int32)
        self.batch, self.lr = batch, lr
        self.h = lib().pdnn_mlp_create(_np_ptr(self.sizes), len(sizes), batch, lr, seed)

    def __del__(self):
        try:
            lib().pdnn_mlp_destroy(self.h)
        except Exception:
            pass

    def weights(self, layer) -> np.ndarray:
        n = lib().pdnn_mlp_layer_size(self.h, layer)
        p = lib().pdnn_mlp_weights(self.h, layer)
        return np.ctypeslib.as_array(p, shape=(n,)).reshape(self.sizes[layer] + 1, self.sizes[layer + 1])

    def grads(self, layer) -> np.ndarray:
        n = lib().pdnn_mlp_layer_size(self.h, layer)
        p = lib().pdnn_mlp_grads(self.h, layer)
        return np.ctypeslib.as_array(p, shape=(n,)).reshape(self.sizes[layer] + 1, self.sizes[layer + 1])

    def forward_backward(self, x: np.ndarray, y: np.ndarray) -> float:
        x = np.ascontiguousarray(x, np.float32)
        y = np.ascontiguousarray(y, np.int32)
        return lib().pdnn_mlp_forward_backward(self.h, _np_ptr(x), _np_ptr(y), len(y))

    def apply(self, lr_scale=1.0):
        lib().pdnn_mlp_apply(self.h, lr_scale)

    def evaluate(self, x, y):
        x = np.ascontiguousarray(x, np.float32)
        y = np.ascontiguousarray(y, np.int32)
        err = ctypes.c_float()
        loss = lib().pdnn_mlp_loss(self.h, _np_ptr(x), _np_ptr(y), len(y), ctypes.byref(err))
        return loss, err.value

    def train(self, x, y, iters):
        x = np.ascontiguousarray(x, np.float32)
        y = np.ascontiguousarray(y, np.int32)
        losses = np.zeros(iters, np.float32)
        lib().pdnn_mlp_train_single(self.h, _np_ptr(x), _np_ptr(y), len(y), iters, _np_ptr(losses))
        return losses


def run_native_role(role, host, port, rank, n_procs, n_to_collect, iters, x, y, sizes, batch=128, lr=1e-3,
                    shortcircuit=True, out_prefix="outfiles/"):
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.int32)
    s = np.asarray(sizes, np.int32)
    if out_prefix:
        os.makedirs(os.path.dirname(out_prefix) or ".", exist_ok=True)
    return lib().pdnn_mlp_run_role(role.encode(), host.encode(), port, rank, n_procs, n_to_collect, iters,
                                   _np_ptr(x), _np_ptr(y), len(y), _np_ptr(s), len(s), batch, lr, int(shortcircuit),
                                   out_prefix.encode())
