"""Work-balanced window sharding and the expected-token estimate (vlog_amd/shard.py), host logic (no GPU)."""
import numpy as np

from vlog_amd.shard import expected_token_order, expected_tokens, partition_by_weight, plan_shards, speech_frames


def test_partition_by_weight_balances_contiguous_ranges():
    rng = np.random.default_rng(0)
    w = rng.uniform(1, 200, size=1200)
    for world in (1, 2, 4, 8):
        parts = partition_by_weight(w, world)
        assert parts[0][0] == 0 and parts[-1][1] == w.size
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        sums = [w[a:b].sum() for a, b in parts]
        assert max(sums) - min(sums) <= 2 * w.max() + 1e-9, (world, sums)


def test_partition_by_weight_skewed_and_tiny():
    w = np.array([100.0] * 10 + [1.0] * 90)          # the work sits in the first tenth
    p = partition_by_weight(w, 2)
    assert p[0][1] <= 10 and p[1] == (p[0][1], 100)
    assert partition_by_weight([5.0, 5.0], 4) == [(0, 1), (1, 2), (2, 2), (2, 2)]
    assert partition_by_weight([], 3) == [(0, 0), (0, 0), (0, 0)]


def test_plan_shards_with_weights_covers_every_window():
    n = 10 * 480000 + 12345
    w = np.arange(11, dtype=np.float64) + 1.0
    plans = plan_shards(n, 3, weights=w)
    assert [p.win0 for p in plans][0] == 0 and plans[-1].win1 == 11
    assert sum(len(p.windows) for p in plans) == 11
    flat = [(p.win0 + i) for p in plans for i in range(len(p.windows))]
    assert flat == list(range(11))


def test_expected_tokens_follow_speech_seconds():
    frame = 512
    db = np.full(30 * 16000 * 3 // frame + 3, -120.0)   # three windows of silence (exact zeros: -inf -> floor)
    db[: 30 * 16000 // frame] = -30.0                    # window 0: all speech
    db[30 * 16000 // frame: 30 * 16000 // frame + 15 * 16000 // frame] = -30.0   # window 1: half
    starts = [0, 480000, 960000]
    t = expected_tokens(db, frame, starts, [480000] * 3)
    assert abs(t[0] - 120.0) < 3 and abs(t[1] - 60.0) < 3 and t[2] == 1.0, t
    assert expected_token_order(t) == [0, 1, 2]
    assert speech_frames(db).sum() == 30 * 16000 // frame + 15 * 16000 // frame
