"""src/merkle_tree/mod.rs on the MI355X: Merkle::commit / batch_commit with
every layer kept on the device (flattened level order, root last)."""
import ctypes

import numpy as np

from .device import check, context, lib, ptr


class Merkle:
    def __init__(self, layers, leaves):
        self.layers_flat = layers  # torch uint8 (2L-1, 32)
        self.num_leaves = leaves
        self._root = None

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
        return t
