"""Optimizer host logic on CPU: the staged update's element ranges (FusedAdam.overlap_with_forward)."""
from distributed_training_and_deepspeed_amd.optim.fused_adam import stage_chunks


def _cover(chunks, n):
    seen = [0] * n
    for rs in chunks:
        for a, b in rs:
            for i in range(a, b):
                seen[i] += 1
    return seen


def test_stage_chunks_cover_buffer_once_with_gaps_and_tied_params():
    # stage 0: [0, 10) and [12, 20); stage 1: [20, 30) and a tied parameter [0, 10) (owned by
    # stage 0, the first span covering it); padding [10, 12) and the tail [30, 35) own no stage
    spans = [(0, 10, 0), (12, 20, 0), (20, 30, 1), (0, 10, 1)]
    ch = stage_chunks(spans, 2, 35)
    assert len(ch) == 3
    assert ch[0] == [(10, 12), (30, 35)]
    assert ch[1] == [(0, 10), (12, 20)]
    assert ch[2] == [(20, 30)]
    assert _cover(ch, 35) == [1] * 35


def test_stage_chunks_merge_adjacent_ranges_and_partial_overlap():
    spans = [(0, 4, 0), (4, 8, 0), (6, 12, 1), (12, 16, 1)]
    ch = stage_chunks(spans, 2, 16)
    assert ch == [[], [(0, 8)], [(8, 16)]]
    assert _cover(ch, 16) == [1] * 16


def test_stage_chunks_no_params():
    assert stage_chunks([], 3, 5) == [[(0, 5)], [], [], []]
