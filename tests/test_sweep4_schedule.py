"""CPU check of the v4 sweep's h_obs schedule (csrc/ame_sweep4.hip).

The natural parameter of node m at slice t sums one observation term per other
node j, with j's NEW mean for j < m and its OLD mean for j > m
(structured_mf.py:289-326, Gauss-Seidel order).  The v4 kernel splits that sum
over four mechanisms that run at different helper steps and read means from
different copies:

  * block GEMM (MFMA) of m's 16-node block b, over j outside the window
    W(b) = [16b - 22, 16b + 16), reading the slice's transposed mean copy Mt
    one step after the loads are issued;
  * window GEMV at helper step m - 2 over j in W(b) minus {m-3 .. m}, reading
    the 64-slot LDS ring of (U, V) rows;
  * HF1 at step m - 1: nodes m - 3 (ring) and m - 2 (the solver's LDS copy);
  * the solver at step m: node m - 1.

This test replays the kernel's timing rules (when each copy of a node's mean
is written, DMA'd, visible, overwritten) and asserts that every (m, j) pair is
covered exactly once and reads the version Gauss-Seidel requires.  The
constants mirror ame_sweep4.hip.
"""
import pytest

BS, GL, GS, MRING, YRING = 16, 22, 18, 64, 8
NGROUP_PER_STEP = 64          # 4 GEMM waves x 16 columns each per step


def window(b, n):
    return max(0, BS * b - GL), min(n, BS * b + BS)


def gemm_load_step(b, j):
    """Helper step at which the GEMM of block b issues the load of column j
    (the part computed at step s is loaded at step s - 1); None = prologue."""
    if b < 2:
        return None
    u = j // 16
    q = (u % NGROUP_PER_STEP) // 4
    return BS * b - GS + q - 1


def mt_new_visible(j, s):
    """Mt[.][j] holds node j's NEW mean for a load issued at step s: written by
    helper wave hw4 at step j + 1, drained at the start of step j + 2, so
    visible after that step's barrier."""
    return s is not None and s >= j + 3


def ring_version(j, s):
    """Version of node j in LDS ring slot j % 64 read at helper step s:
    old row DMA'd at step j - GL (prologue if j < GL, usable 3 steps later),
    new row written at step j + 1 (usable from j + 2)."""
    dma = j - GL
    usable_old = -1 if dma < 0 else dma + 3
    if s >= j + 2:
        # slot must not have been re-filled by node j + 64's old row yet
        assert s < (j + 64 - GL) + 1, (j, s)
        return "new"
    assert s >= usable_old, f"old row of node {j} not landed at step {s}"
    assert s < j + 1 or s >= j + 2
    return "old"


@pytest.mark.parametrize("n", [8, 16, 20, 36, 64, 100, 256, 1024, 1040, 2048])
def test_every_pair_covered_once_with_the_right_version(n):
    for m in range(n):
        b = m // BS
        lo, hi = window(b, n)
        seen = {}
        for j in range(n):
            if j == m:
                continue
            want = "new" if j < m else "old"
            got = []
            if not (lo <= j < hi):
                s = gemm_load_step(b, j)
                if s is None:   # prologue GEMM of blocks 0, 1: every mean is old
                    assert j >= m, (m, j)
                    got.append("old")
                else:
                    assert s >= -1
                    got.append("new" if mt_new_visible(j, s) else "old")
                    # a column that is still old must not be overwritten before
                    # the load (written at step j + 1 at the earliest)
            else:
                if j <= m - 4 or j >= m + 1:
                    got.append(ring_version(j, m - 2) if m >= 2 else "old")
                elif j in (m - 3, m - 2):
                    got.append("new")      # HF1 at step m - 1
                elif j == m - 1:
                    got.append("new")      # solver at step m
            assert len(got) == 1, (m, j, got)
            assert got[0] == want, (n, m, j, got[0], want)
            seen[j] = True
        assert len(seen) == n - 1


@pytest.mark.parametrize("n", [64, 1024, 2048])
def test_block_results_live_long_enough(n):
    """H_blk[b & 1] is reduced at step 16b - 2, read by HF1 at steps
    [16b - 1, 16b + 15), and overwritten by block b + 2 at step 16b + 30."""
    for b in range(2, (n + BS - 1) // BS):
        red = BS * b - 2
        first_use, last_use = BS * b - 1, min(n, BS * b + BS) - 2
        assert red < first_use
        assert BS * (b + 2) - 2 > last_use
        # the GEMM of block b finished its last part at step 16b - 3
        assert BS * b - GS + 15 == red - 1


def test_y_window_ring():
    """Y window of row m: DMA at step m - 5 (usable at m - 2), read at steps
    m - 2 (window GEMV), m - 1 (HF1), m (solver); slot m % 8 is refilled for
    row m + 8 at step m + 3."""
    for m in range(5, 200):
        assert (m - 5) + 3 <= m - 2
        assert (m + 8) - 5 > m
        lo, hi = window(m // BS, 10 ** 6)
        assert lo <= m - 3 and hi - lo <= 128      # 128 float2 per 1-KiB slot
