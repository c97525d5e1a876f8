"""Transcript (src/transcript.rs) over the C ABI (host SHA-256 in libmlhip)."""
import ctypes

from .device import check, fe_from_bytes, lib


class Transcript:
    """transcript.rs:5-38: running SHA-256; random() finalizes a clone;
    next_challenge() = F::from(u128_le(random()[..16])) without absorbing."""

    def __init__(self, _handle=None):
        if _handle is None:
            h = ctypes.c_void_p()
            check(lib().mlh_transcript_create(ctypes.byref(h)))
            _handle = h.value
        self.h = _handle

    def __del__(self):
        try:
            lib().mlh_transcript_destroy(self.h)
        except Exception:
            pass

    def clone(self):
        h = ctypes.c_void_p()
        check(lib().mlh_transcript_clone(self.h, ctypes.byref(h)))
        return Transcript(h.value)

    def absorb(self, data: bytes):
        buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data) if data else None
        check(lib().mlh_transcript_absorb(self.h, buf, len(data)))

    def random(self) -> bytes:
        out = (ctypes.c_uint8 * 32)()
        check(lib().mlh_transcript_random(self.h, out))
        return bytes(out)

    def next_challenge(self) -> int:
        out = (ctypes.c_uint8 * 16)()
        check(lib().mlh_transcript_next_challenge(self.h, out))
        return fe_from_bytes(out)
