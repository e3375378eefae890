"""bench.py's reporting logic without a GPU: the C4 blocks' per-stage
maximum over ranks (a SCALE run must show which rank bounds
each stage) with fake ranks, and the per-rank frame counts of the shard."""
import math

from bench import C4_STAGES, c4_stage_table
from vcf_amd.codec.shard import frame_range


def test_stage_maxima_over_fake_ranks():
    world, N = 8, 256
    rows = [[0.001 * (s + 1) + 0.0001 * r * (1 if s % 2 else -1) for r in range(world)] for s in range(len(C4_STAGES))]
    fpr = [frame_range(N, r, world)[1] - frame_range(N, r, world)[0] for r in range(world)]
    t = c4_stage_table(rows, fpr)
    assert t["frames_per_rank"] == [32] * 8 and sum(t["frames_per_rank"]) == N
    for s, name in enumerate(C4_STAGES):
        want = max(rows[s])
        assert math.isclose(t["stages_ms_max"][name], round(want * 1e3, 3))
        assert t["slowest_rank"][name] == (world - 1 if s % 2 else 0)
        assert math.isclose(t["stages_ms_rank0"][name], round(rows[s][0] * 1e3, 3))


def test_stage_table_skips_missing_ranks():
    nan = float("nan")
    rows = [[nan, 0.002, 0.003]] + [[nan, nan, nan]] * (len(C4_STAGES) - 1)
    t = c4_stage_table(rows, [3, 3, 2])
    assert t["stages_ms_max"] == {C4_STAGES[0]: 3.0} and t["slowest_rank"] == {C4_STAGES[0]: 2}
    assert t["stages_ms_rank0"] == {}


def test_c3_fp64_op_count():
    """C3's float64 work per pixel: bior4.4 (9 + 7 nonzero decomposition taps)
    gives 30 multiplies + adds per output pair, two passes per level, three
    channels, five levels of planes a quarter the size: 90 * (1 + 1/4 + ... + 1/256)."""
    import bench
    assert abs(bench.c3_fp64_ops_per_pixel() - 90 * sum(0.25 ** l for l in range(5))) < 1e-9
    assert abs(bench.c3_fp64_ops_per_pixel(levels=1) - 90.0) < 1e-9
