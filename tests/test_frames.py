"""Multi-frame launcher (webgputracer_amd/frames.py): frame range semantics and the
partition over ranks (CPU).  `--frame s e` renders the frame indices s-1 ... e-1
(render.cpp:437-439) and names them "%03d.png" % i (render.cpp:493-497)."""
import pytest

from webgputracer_amd.frames import batches, frame_indices, frames_of_rank, main


def test_frame_indices_follow_oncompute_loop():
    # for (uint32_t i = start_frame - 1; i < end_frame; ++i) OnRender(i);
    assert frame_indices(1, 1) == [0]
    assert frame_indices(1, 600) == list(range(0, 600))
    assert frame_indices(321, 600) == list(range(320, 600))  # settings/run.py:22
    assert frame_indices(1, 320) + frame_indices(321, 600) == frame_indices(1, 600)  # run.py:11 + :22
    assert frame_indices(3, 2) == [] and frame_indices(0, 5) == []


@pytest.mark.parametrize("start,end", [(1, 600), (1, 1), (5, 9), (321, 600)])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_frames_partition_range(start, end, world):
    """Every frame of the range lands on exactly one rank; shares differ by <= 1."""
    shares = [frames_of_rank(start, end, r, world) for r in range(world)]
    flat = sorted(f for s in shares for f in s)
    assert flat == list(range(start - 1, end))
    assert max(map(len, shares)) - min(map(len, shares)) <= 1


def test_batches_cover_in_order():
    fr = frames_of_rank(1, 23, 1, 4)
    bs = batches(fr, 4)
    assert [f for b in bs for f in b] == fr
    assert all(1 <= len(b) <= 4 for b in bs)
    assert frames_of_rank(3, 2, 0, 1) == []


@pytest.mark.parametrize("rng", [["0", "3"], ["4", "3"]])
def test_bad_frame_range_rejected(rng):
    """Same check as the C++ CLI (csrc/main.cpp): start >= 1, end >= start."""
    with pytest.raises(SystemExit):
        main(["--frame", *rng])
