"""Host-side checks of the persistent decode tail (csrc/kernels/mlp_engine.hip): the kernel's own work-split
function (exported for this test) hands every activation group and every down-row group to exactly one
workgroup for any grid size, within the per-workgroup LDS partial capacity the shape gate promises."""
import ctypes

import pytest

from rag_llm_k8s_amd.ops import _lib

ME_KC, ME_MAXA, ME_MAXB = 512, 64, 56


def _split(G, H, I):
    L = _lib.lib()
    out = (ctypes.c_int * 4)()
    rows = []
    for w in range(G):
        assert L.ragk_mlp_engine_split(G, w, H, I, ctypes.cast(out, ctypes.c_void_p)) == 0
        rows.append(tuple(out))
    return rows


@pytest.mark.parametrize("G", [256, 304, 240, 80, 8, 1])
@pytest.mark.parametrize("H,I", [(4096, 14336), (1024, 2048), (2048, 5632)])
def test_split_covers_every_group_once(G, H, I):
    rows = _split(G, H, I)
    NA, ND = I // 8, H // 16
    assert rows[0][0] == 0 and rows[-1][1] == NA and rows[0][2] == 0 and rows[-1][3] == ND
    for (a0, a1, d0, d1), nxt in zip(rows, rows[1:] + [None]):
        assert a0 <= a1 and d0 <= d1
        if nxt is not None:
            assert nxt[0] == a1 and nxt[2] == d1  # contiguous, no gap, no overlap
    ok = _lib.lib().ragk_mlp_engine_ok(1, H, I, G)
    fits = all((a1 - a0) * (H // ME_KC) <= ME_MAXA and (d1 - d0) * (I // ME_KC) <= ME_MAXB
               and (a1 - a0) * 8 <= 64 and (d1 - d0) * 16 <= 64 for a0, a1, d0, d1 in rows)
    if ok:  # the shape gate never admits a grid whose split overflows the partial-sum capacity
        assert fits


def test_split_weights_even_and_odd_xcds():
    """Llama-3.1-8B on 256 CUs: workgroups on even XCDs (w % 8 even) get 6 activation groups, those on odd
    XCDs 8 (the measured per-XCD stream rates: even ~15 % slower)."""
    rows = _split(256, 4096, 14336)
    even = sum(r[1] - r[0] for w, r in enumerate(rows) if w % 2 == 0)
    odd = sum(r[1] - r[0] for w, r in enumerate(rows) if w % 2 == 1)
    assert even + odd == 14336 // 8
    assert all(r[1] - r[0] == (6 if w % 2 == 0 else 8) for w, r in enumerate(rows))
    assert _lib.lib().ragk_mlp_engine_ok(1, 4096, 14336, 256)
