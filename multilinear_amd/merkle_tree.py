"""src/merkle_tree/mod.rs on the MI355X: Merkle::commit / batch_commit with
every layer kept on the device (flattened level order, root last)."""
import ctypes

import numpy as np

from . import _lib
from .device import check, context, lib, ptr

LEFT = 0  # Direction::Left (merkle_tree/mod.rs:14-17)
RIGHT = 1


class Merkle:
    def __init__(self, layers, leaves):
        self.layers_flat = layers  # torch uint8 (2L-1, 32)
        self.num_leaves = leaves
        self._root = None
        self._item = None  # index -> opened value (bytes, or list of bytes for batches)
        self.device = layers.device.index or 0

    def _siblings(self, index):
        if index < 0 or index >= self.num_leaves:
            return None
        depth = self.num_leaves.bit_length() - 1
        idx = (ctypes.c_uint64 * 1)(index)
        out = (ctypes.c_uint8 * max(1, 32 * depth))()
        ctx = context(self.device)
        check(lib().mlh_merkle_open(ctx, ptr(self.layers_flat), self.num_leaves, idx, 1, out), ctx)
        raw = bytes(out)
        return [(raw[32 * i:32 * i + 32], LEFT if (index >> i) & 1 else RIGHT)
                for i in range(depth)]

    def open(self, index):
        """Merkle::open (merkle_tree/mod.rs:31-58) -> (value, [(sibling, direction)]),
        or None past the last leaf."""
        path = self._siblings(index)
        if path is None:
            return None
        return (self._item(index) if self._item else None), path

    def batch_open(self, index):
        """Merkle::batch_open (merkle_tree/mod.rs:134-175): the column of the
        batches at `index` and its path."""
        return self.open(index)

    def root(self) -> bytes:
        """merkle_tree/mod.rs:27-29."""
        return bytes(self._root)

    def layers(self):
        """list of numpy (len, 32) uint8 arrays, leaves first (Merkle::layers)."""
        flat = self.layers_flat.cpu().numpy()
        out, off, n = [], 0, self.num_leaves
        while n >= 1:
            out.append(flat[off:off + n])
            off += n
            if n == 1:
                break
            n //= 2
        return out

    @staticmethod
    def _alloc(leaves, device):
        import torch

        return torch.empty((2 * leaves - 1, 32), dtype=torch.uint8, device="cuda:%d" % device)

    @staticmethod
    def commit_pairs(code, device=0):
        """commit_rs_code (fri/mod.rs:45-55): leaves (code[i], code[i+n/2])."""
        n = code.shape[0]
        ctx = context(device)
        t = Merkle(Merkle._alloc(n // 2, device), n // 2)
        root = (ctypes.c_uint8 * 32)()
        check(lib().mlh_merkle_commit_pairs(ctx, ptr(code), n.bit_length() - 1, ptr(t.layers_flat),
                                            root), ctx)
        t._root = root
        # ReedSolomonPair bytes LE16(code[i]) || LE16(code[i + n/2]) (fri/mod.rs:30-43)
        t._item = lambda i: (code[i].cpu().numpy().tobytes() +
                             code[i + n // 2].cpu().numpy().tobytes())
        return t

    @staticmethod
    def commit(items, device=0):
        """Merkle::commit (merkle_tree/mod.rs:65-85) over equal-length byte items."""
        import torch

        items = [bytes(x) for x in items]
        n = len(items)
        ln = len(items[0])
        assert all(len(x) == ln for x in items)
        dev = torch.from_numpy(np.frombuffer(b"".join(items), dtype=np.uint8).copy()).to(
            "cuda:%d" % device)
        ctx = context(device)
        t = Merkle(Merkle._alloc(n, device), n)
        root = (ctypes.c_uint8 * 32)()
        check(lib().mlh_merkle_commit(ctx, ptr(dev), ln, n, ptr(t.layers_flat), root), ctx)
        t._root = root
        t._item = lambda i: dev[i * ln:(i + 1) * ln].cpu().numpy().tobytes()
        return t

    @staticmethod
    def batch_commit(batches, device=0):
        """Merkle::batch_commit (merkle_tree/mod.rs:92-131)."""
        import torch

        m = len(batches)
        n = len(batches[0])
        ln = len(bytes(batches[0][0]))
        raw = b"".join(bytes(x) for b in batches for x in b)
        dev = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to("cuda:%d" % device)
        ctx = context(device)
        t = Merkle(Merkle._alloc(n, device), n)
        root = (ctypes.c_uint8 * 32)()
        check(lib().mlh_merkle_batch_commit(ctx, ptr(dev), ln, m, n, ptr(t.layers_flat), root), ctx)
        t._root = root
        t._item = lambda i: [dev[(j * n + i) * ln:(j * n + i + 1) * ln].cpu().numpy().tobytes()
                             for j in range(m)]
        return t


def verify_status(value, path, root, index):
    """MerkleInclusionPath::verify (merkle_tree/mod.rs:216-253) on the host
    (libmlhip): MLH_OK, MLH_ERR_VERIFY (IncompatibleHash) or
    MLH_ERR_VERIFY_INDEX (IncompatibleIndex).  value: bytes, or a list of
    items (batch_verify, :255-293, hashes their concatenation)."""
    if isinstance(value, (list, tuple)):
        value = b"".join(bytes(v) for v in value)
    value = bytes(value)
    sibs = b"".join(bytes(sib) for sib, _ in path)
    dirs = sum(1 << i for i, (_, d) in enumerate(path) if d == LEFT)
    vb = (ctypes.c_uint8 * max(1, len(value))).from_buffer_copy(value or b"\0")
    sb = (ctypes.c_uint8 * max(1, len(sibs))).from_buffer_copy(sibs or b"\0")
    rb = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(root))
    return lib().mlh_merkle_verify(vb, len(value), sb, len(path), dirs, rb, index)


def verify(value, path, root, index):
    """True iff verify / batch_verify returns Ok(())."""
    return verify_status(value, path, root, index) == _lib.MLH_OK


batch_verify = verify
