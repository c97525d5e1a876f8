"""SHA-256 Merkle tree (oracle).  Test infrastructure only.

Reference: src/merkle_tree/mod.rs.  Leaves are hash_leaf(item bytes)
(:178-182); nodes hash_node(left ‖ right) (:184-189); every layer kept,
layers[0] = leaf digests, root = layers[-1][0] (:27-29, :65-85).
"""
import hashlib


def hash_leaf(item: bytes) -> bytes:  # merkle_tree/mod.rs:178-182
    return hashlib.sha256(item).digest()


def hash_node(left: bytes, right: bytes) -> bytes:  # merkle_tree/mod.rs:184-189
    return hashlib.sha256(left + right).digest()


class Merkle:
    def __init__(self, layers, data):
        self.layers = layers
        self.data = data

    @staticmethod
    def commit(data):
        """Merkle::commit (merkle_tree/mod.rs:65-85); data = list of bytes."""
        n = len(data)
        assert n > 0 and n & (n - 1) == 0, "Data length must be a power of two"
        layers = [[hash_leaf(d) for d in data]]
        while len(layers[-1]) > 1:
            cur = layers[-1]
            layers.append([hash_node(cur[2 * i], cur[2 * i + 1]) for i in range(len(cur) // 2)])
        return Merkle(layers, data)

    @staticmethod
    def batch_commit(data):
        """Merkle::batch_commit (merkle_tree/mod.rs:92-131): leaf i =
        SHA256(data[0][i] ‖ data[1][i] ‖ ...)."""
        assert data, "Data must not be empty"
        n = len(data[0])
        assert n & (n - 1) == 0
        assert all(len(b) == n for b in data)
        first = [hashlib.sha256(b"".join(b[i] for b in data)).digest() for i in range(n)]
        layers = [first]
        while len(layers[-1]) > 1:
            cur = layers[-1]
            layers.append([hash_node(cur[2 * i], cur[2 * i + 1]) for i in range(len(cur) // 2)])
        return Merkle(layers, data)

    def root(self) -> bytes:  # merkle_tree/mod.rs:27-29
        return self.layers[-1][0]

    def open(self, index):
        """Merkle::open (merkle_tree/mod.rs:31-58) -> (value, [(sibling, dir)])
        dir: 0 = Left (sibling on the left), 1 = Right."""
        if index >= len(self.data):
            return None
        path = []
        cur = index
        for layer in self.layers:
            if cur % 2 == 0:
                sib, d = cur + 1, RIGHT
            else:
                sib, d = cur - 1, LEFT
            if sib >= len(layer):
                break
            path.append((layer[sib], d))
            cur //= 2
        assert len(path) == len(self.layers) - 1
        return (self.data[index], path)


LEFT = 0  # Direction::Left  (merkle_tree/mod.rs:14-17, repr(u8))
RIGHT = 1


def verify(value: bytes, path, root: bytes, index: int) -> bool:
    """MerkleInclusionPath::verify (merkle_tree/mod.rs:216-253)."""
    h = hashlib.sha256(value).digest()
    computed_index = 0
    for i, (sib, d) in enumerate(path):
        if d == LEFT:
            computed_index += 1 << i
            h = hash_node(sib, h)
        else:
            h = hash_node(h, sib)
    return h == root and computed_index == index


def batch_open(tree, index):
    """Merkle::batch_open (merkle_tree/mod.rs:134-175): the column
    data[j][index] for every batch j, and the sibling path."""
    if index >= len(tree.data[0]):
        return None
    value = [b[index] for b in tree.data]
    path = []
    cur = index
    for layer in tree.layers:
        sib, d = (cur + 1, RIGHT) if cur % 2 == 0 else (cur - 1, LEFT)
        if sib >= len(layer):
            break
        path.append((layer[sib], d))
        cur //= 2
    return value, path


def batch_verify(value, path, root, index):
    """MerkleInclusionPath::batch_verify (merkle_tree/mod.rs:255-293)."""
    return verify(b"".join(value), path, root, index)
