"""Multi-frame launcher (webgputracer_amd/frames.py): frame partition over ranks (CPU)."""
import pytest

from webgputracer_amd.frames import batches, frames_of_rank


@pytest.mark.parametrize("start,end", [(1, 600), (1, 1), (5, 9), (321, 600)])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_frames_partition_range(start, end, world):
    """Every frame of [start, end] lands on exactly one rank; shares differ by <= 1
    (settings/run.py splits 1-320 / 321-600 over two machines)."""
    shares = [frames_of_rank(start, end, r, world) for r in range(world)]
    flat = sorted(f for s in shares for f in s)
    assert flat == list(range(start, end + 1))
    assert max(map(len, shares)) - min(map(len, shares)) <= 1


def test_batches_cover_in_order():
    fr = frames_of_rank(1, 23, 1, 4)
    bs = batches(fr, 4)
    assert [f for b in bs for f in b] == fr
    assert all(1 <= len(b) <= 4 for b in bs)
    assert frames_of_rank(3, 2, 0, 1) == []
