"""bench.py's launch and timed-region plan, on the CPU (no GPU):

* the encoder plan of the driver's command lines (--steps 1 / 7 / 20 / 120,
  --warmup 5, the default encoder batch 8 and 8 frames ahead, and other
  lookahead settings): exactly `steps` image encodes are queued by the timed
  steps, each replay holds at most enc_batch images, every frame is encoded
  exactly once, and the frames the bench allocates suffice;
* `--gpus 2` without an external launcher spawns two ranks that meet over
  gloo (--dist-dry-run), shard a pair list and report world size and backend.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


@pytest.mark.parametrize("steps", [1, 7, 20, 120])
@pytest.mark.parametrize("kb,ahead", [(8, 8), (1, None), (4, 4), (8, None), (3, 5)])
def test_timed_region_holds_exactly_steps_encodes(steps, kb, ahead):
    warmup = 5
    p = bench.plan_encodes(steps, warmup, kb, ahead)
    assert p["timed_encodes"] == steps
    assert all(1 <= c <= kb for _, c, _ in p["batches"])
    # every frame encoded once, in order, no gaps
    frames = [s + j for s, c, _ in p["batches"] for j in range(c)]
    assert frames == list(range(len(frames)))
    # every stepped frame is encoded (frames 0 .. warmup + steps)
    assert len(frames) >= warmup + steps + 1
    # lookahead images past the bench's 16-frame tail repeat its last frame
    assert p["frames_needed"] <= warmup + steps + 1 + 33
    # timed replays come after every warm-up replay
    flags = [t for _, _, t in p["batches"]]
    assert flags == sorted(flags)


def test_driver_command_plan_has_a_partial_last_batch():
    p = bench.plan_encodes(20, 5, 8, 8)
    timed = [(s, c) for s, c, t in p["batches"] if t]
    assert sum(c for _, c in timed) == 20
    assert any(c < 8 for _, c in timed)


def test_no_pipeline_encodes_each_frame_in_its_step():
    p = bench.plan_encodes(20, 5, 8, 8, pipeline=False)
    assert p["timed_encodes"] == 20
    assert all(c == 1 for _, c, _ in p["batches"])


def test_frontend_rule_matches_the_plan():
    """slam.lookahead_batches (the Frontend's rule) drives the simulation:
    batches of at most enc_batch until frame i + enc_ahead is queued, a
    partial batch when fewer images are handed over."""
    from splatt3r_amd.slam import lookahead_batches
    assert lookahead_batches(5, 6, 16, 8, 8) == [(6, 8)]          # frames up to 13 queued
    assert lookahead_batches(5, 6, 16, 8, 9) == [(6, 8), (14, 8)]
    assert lookahead_batches(0, 1, 3, 8, 8) == [(1, 3)]
    assert lookahead_batches(0, 1, 0, 8, 8) == []
    assert lookahead_batches(10, 30, 16, 8, 8) == []
    assert lookahead_batches(3, 4, 16, 1, None) == [(4, 1)]


def test_gpus_flag_spawns_ranks_without_a_launcher():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--dist-dry-run"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["world_size"] == 2 and d["n_gpus"] == 2 and d["dist_backend"] == "gloo"
    assert d["pairs_covered"] == d["pairs"]
    # the sharded backend leg's protocol: rank 0's worker thread + PairShard,
    # rank 1 in serve_backend; every pair's two directed units ran somewhere
    be = d["backend"]
    assert be["keyframes"] == 9 and be["edges"] == be["pairs"] > 0
    assert be["units_all_ranks"] == 2 * be["pairs"] and 0 < be["rank0_units"] < 2 * be["pairs"]
    # the sharded-unit self-check the GPU run prints (shard_check): units and
    # map edges produced on rank 1, re-decoded on rank 0, equal bit for bit
    sc = d["shard_check"]
    assert sc["equal"] is True
    assert sc["pairs"]["units"] and all(u["rank"] == 1 for u in sc["pairs"]["units"])
    assert sc["map"]["edges"] and all(e["rank"] == 1 for e in sc["map"]["edges"])


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--dist-dry-run"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_driver_plan_overlaps_every_timed_replay():
    """The driver's plan queues every timed encoder replay enc_ahead frames
    before its first frame (the steady state's lead: no timed frame waits for
    its encode) and the last one before the last timed step, so that no
    replay runs alone after the last tracked frame."""
    from splatt3r_amd.slam import lookahead_batches
    steps, warmup, kb, ahead = 20, 5, 8, 8
    p = bench.plan_encodes(steps, warmup, kb, ahead)
    assert p["timed_encodes"] == steps
    # replay the frontend's rule with the plan's caps to get the queuing steps
    look = p["look"]
    nxt_enc, queued = p["next_enc_before"], []
    for i in range(warmup + 1, warmup + steps + 1):
        hi = min(i + 1 + look, p["cap"])
        for s, c in lookahead_batches(i, nxt_enc, max(0, hi - (i + 1)), kb, ahead):
            queued.append((i, s, c))
            nxt_enc = s + c
    assert sum(c for _, _, c in queued) == steps
    assert all(s - i >= ahead for i, s, _ in queued)
    assert queued[-1][0] < warmup + steps
