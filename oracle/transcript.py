"""Fiat-Shamir transcript (oracle).  Test infrastructure only.

Reference: src/transcript.rs:5-55.  A running SHA-256 (sha2 0.10.8; the
published FIPS 180-4 algorithm, restated here by hashlib).
"""
import hashlib

from . import field as F


class Transcript:
    def __init__(self):  # transcript.rs:17-21
        self.state = hashlib.sha256()

    def clone(self):
        t = Transcript()
        t.state = self.state.copy()
        return t

    def random(self) -> bytes:
        """transcript.rs:23-29: finalize a clone, state unchanged."""
        return self.state.copy().digest()

    def absorb(self, data: bytes):  # transcript.rs:31-33
        self.state.update(data)

    def next_challenge(self) -> int:
        """transcript.rs:35-38: F::from(u128_le(random()[0..16])); no absorb."""
        return F.from_u128(int.from_bytes(self.random()[:16], "little"))
