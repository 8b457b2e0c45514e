"""Paged KV-cache block manager (64-token blocks).

Uses the native C++ allocator from ``_ragk_rt`` when built (O(1) free-list ops in C++,
called once per scheduled sequence per step); the Python class below has the identical
interface and is the fallback / test oracle.

Block 0 is reserved as a scratch block: padded (dummy) rows of a captured decode graph
write their K/V there, so graph replay never touches a live sequence's cache.
"""
from __future__ import annotations

BLOCK = 64


class PyBlockManager:
    def __init__(self, num_blocks: int, reserve_scratch: bool = True):
        if num_blocks < 2:
            raise ValueError("need at least 2 KV blocks")
        self.num_blocks = num_blocks
        self.scratch = 0 if reserve_scratch else -1
        first = 1 if reserve_scratch else 0
        self._free = list(range(num_blocks - 1, first - 1, -1))
        self.tables = {}

    def free_blocks(self) -> int:
        return len(self._free)

    def blocks_needed(self, seq_id, n_tokens) -> int:
        have = len(self.tables.get(seq_id, ()))
        need = -(-n_tokens // BLOCK)
        return max(0, need - have)

    def can_allocate(self, seq_id, n_tokens) -> bool:
        return self.blocks_needed(seq_id, n_tokens) <= len(self._free)

    def ensure(self, seq_id, n_tokens):
        """Make sure the sequence owns blocks for positions [0, n_tokens). Returns the table."""
        t = self.tables.setdefault(seq_id, [])
        need = -(-n_tokens // BLOCK)
        if need - len(t) > len(self._free):
            raise MemoryError("KV cache exhausted")
        while len(t) < need:
            t.append(self._free.pop())
        return t

    def table(self, seq_id):
        return self.tables.get(seq_id, [])

    def slot(self, seq_id, pos) -> int:
        return self.tables[seq_id][pos // BLOCK] * BLOCK + pos % BLOCK

    def free(self, seq_id):
        t = self.tables.pop(seq_id, None)
        if t:
            self._free.extend(reversed(t))


def make_block_manager(num_blocks: int):
    try:
        from ..runtime import native_rt

        rt = native_rt()
        if rt is not None:
            return rt.BlockManager(num_blocks, True)
    except Exception:
        pass
    return PyBlockManager(num_blocks)
