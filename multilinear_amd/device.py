"""Device plumbing: the mlhip context, torch-allocated HBM buffers, and
conversions between Python ints / numpy limb arrays / device tensors.

A field vector on the device is a contiguous ``torch.int32`` tensor of shape
(n, 4): four little-endian u32 limbs of the canonical u128 -- byte for byte
the reference's ``Vec<Field128>`` (src/field.rs:33-38).  torch is used only
for memory, streams and torch.distributed; all arithmetic runs in libmlhip.
"""
import ctypes

import numpy as np

from . import _lib

M = 340282366920938463463374557953744961537

_ctx = {}


def lib():
    return _lib.load()


def check(status, ctx=None):
    if status != _lib.MLH_OK:
        msg = ""
        if ctx is not None:
            msg = (lib().mlh_last_error(ctx) or b"").decode()
        raise _lib.MlhError(status, msg)


def context(device=0):
    """The per-device mlhip context, bound to torch's current HIP stream."""
    import torch

    st = torch.cuda.current_stream(device).cuda_stream
    c = _ctx.get(device)
    if c is None:
        h = ctypes.c_void_p()
        st_ = lib().mlh_context_create(device, ctypes.c_void_p(st), ctypes.byref(h))
        if st_ != _lib.MLH_OK:
            raise _lib.MlhError(st_, (lib().mlh_last_error(None) or b"").decode())
        c = h.value
        _ctx[device] = c
    else:
        lib().mlh_set_stream(c, ctypes.c_void_p(st))
    return c


# ---- conversions -----------------------------------------------------------

def ints_to_limbs(values):
    """list of ints in [0, 2^128) -> (n, 4) uint32 little-endian limbs."""
    b = b"".join(int(v).to_bytes(16, "little") for v in values)
    return np.frombuffer(b, dtype=np.uint32).reshape(-1, 4).copy()


def limbs_to_ints(arr):
    a = np.ascontiguousarray(arr, dtype=np.uint32).reshape(-1, 4)
    raw = a.tobytes()
    return [int.from_bytes(raw[16 * i:16 * i + 16], "little") for i in range(a.shape[0])]


def fe_bytes(v):
    return (ctypes.c_uint8 * 16).from_buffer_copy(int(v).to_bytes(16, "little"))


def fe_from_bytes(b):
    return int.from_bytes(bytes(b), "little")


def to_device(limbs, device=0):
    import torch

    a = np.ascontiguousarray(limbs, dtype=np.uint32).reshape(-1, 4)
    return torch.from_numpy(a.view(np.int32)).to("cuda:%d" % device)


def from_device(t):
    return t.detach().cpu().contiguous().numpy().view(np.uint32).reshape(-1, 4)


def empty(n, device=0):
    import torch

    return torch.empty((n, 4), dtype=torch.int32, device="cuda:%d" % device)


def random_limbs(n, seed):
    """Seeded uniform canonical elements (top limb < 0xFFFFFFFF => < M)."""
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 2**32, size=(n, 4), dtype=np.uint64).astype(np.uint32)
    a[:, 3] = np.minimum(a[:, 3], np.uint32(0xFFFFFFFE))
    return a


def random_device(n, seed, device=0):
    """Uniform canonical elements generated on the device (torch RNG)."""
    import torch

    g = torch.Generator(device="cuda:%d" % device)
    g.manual_seed(seed)
    t = torch.randint(-(2**31), 2**31, (n, 4), dtype=torch.int32, device="cuda:%d" % device,
                      generator=g)
    # clear bit 0 of the top limb's... force top limb <= 0xFFFFFFFE: top != -1
    top = t[:, 3]
    t[:, 3] = torch.where(top == -1, torch.zeros_like(top), top)
    return t


def ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class ntt_plan:
    """Context manager forcing the NTT radix plan of this device's context
    (mlh_set_ntt_plan), e.g. ``with ntt_plan("9,4,4"): ...`` -- test/tuning hook."""

    def __init__(self, plan, device=0):
        self.digits = [int(v) for v in plan.split(",")] if isinstance(plan, str) else list(plan)
        self.device = device

    def __enter__(self):
        import ctypes

        ctx = context(self.device)
        arr = (ctypes.c_uint32 * len(self.digits))(*self.digits)
        check(lib().mlh_set_ntt_plan(ctx, arr, len(self.digits)), ctx)
        return self

    def __exit__(self, *exc):
        ctx = context(self.device)
        check(lib().mlh_set_ntt_plan(ctx, None, 0), ctx)
        return False
