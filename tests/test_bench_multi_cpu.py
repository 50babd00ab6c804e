"""bench.py's JSON line at N > 1 (VERDICT r4 Next #1): after the data-parallel headline, the timed
multi-GPU blocks — ``rccl_search`` (C1 + C2 as collectives, >= 3 timed sharded searches here, rows
identical to the serving plane), ``serving_search`` (the owner-routed serving plane vs the
SEARCH_TRANSPORT=rccl collective rounds under a serving load, same ids), ``tp_decode`` (the decoder at TP = N, decode ms per step at batch 1
and batch B per all-reduce arm, the per-decision TP verdict) — plus the single-document ingest
latency and the physical-GPU count. Rehearsed on CPU ranks (gloo, tiny configs): the schema and the
verdicts are pinned here; the numbers come from the GPU node."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_rank_json_schema():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-rehearsal",
           "--enc", "tiny-enc", "--llm", "tiny-dec", "--batch", "2", "--steps", "1", "--warmup", "0",
           "--latency-reps", "2", "--ingest-docs", "2", "--ingest-batches", "1", "--ingest-latency-reps", "2",
           "--index-rows", "2000", "--multi-iters", "3", "--breakdown", "0", "--max-new", "4",
           "--ingest-words", "300", "--serving-requests", "12",
           # the 70B block's code path on a miniature of its TP = 8 layout
           "--tp70b", "on", "--tp70b-arch", "tiny-dec-tp8", "--tp70b-batches", "1,2"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    # driver contract + the physical-device count (two CPU ranks share this host: not two GPUs)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["world_size"] == 2 and out["ranks_seen"] == 2
    assert out["n_gpus"] == 1 and out["oversubscribed"] is True
    # the QA steps' search ran as the lock-step collective (C2 + C1), not over the host plane
    assert out["config"]["search_transport"].startswith("rccl"), out["config"]
    # the reference's ingest number: per-document latency
    assert out["ingest_single_doc_reps"] == 2 and out["ingest_single_doc_p50_ms"] > 0
    # C1 + C2 over the collective backend, timed, identical rows to the plane
    rs = out["rccl_search"]
    assert rs["iters"] == 3 and rs["rows_per_rank"] == 2 and rs["world"] == 2, rs
    assert rs["qps"] > 0 and rs["p50_ms"] > 0 and rs["p90_ms"] >= rs["p50_ms"], rs
    assert rs["rows_identical_to_plane"] == rs["rows_checked"] == 2 and rs["scores_close"], rs
    # the serving transports under load: owner-routed plane vs lock-step collective rounds, same ids
    ss = out["serving_search"]
    assert "error" not in ss, ss
    assert ss["requests_per_rank"] == 12 and ss["ids_identical"] is True and ss["rounds"] >= 1, ss
    for t in ("plane", "rccl"):
        assert ss[t]["searches_per_s"] > 0 and ss[t]["p90_ms"] >= ss[t]["p50_ms"] > 0, ss
    # TP = N decode per arm, batch 1 and batch B, plus the agreement verdict
    td = out["tp_decode"]
    assert td["tp"] == 2 and "error" not in td, td
    assert td["arms"], td
    for arm in td["arms"].values():
        assert arm["b1_decode_ms_per_step"] > 0 and arm["b2_decode_ms_per_step"] > 0, td
    ag = td["agreement"]
    assert ag["ok"] and ag["checked_agree"] == ag["checked"] > 0, ag
    # gloo has no graph-captured collective arm; every arm timed both batches
    assert "rccl_graph" not in td["arms"] and "gloo_eager" in td["arms"], td
    # BASELINE config 5's QA model block: built as TP = N shards (no unsharded weights), timed per batch
    t7 = out["tp_decode_70b"]
    assert "error" not in t7 and t7["tp"] == 2 and t7["model"] == "tiny-dec-tp8", t7
    assert "agreement" not in t7 and list(t7["arms"]) == ["gloo_eager"], t7
    for arm in t7["arms"].values():
        assert arm["b1_decode_ms_per_step"] > 0 and arm["b2_decode_ms_per_step"] > 0 and arm["b2_prefill_ms"] > 0, t7
    # per-rank HBM plan per phase (parallel/hbm_plan.py); peaks are GPU-only
    assert set(out["hbm_plan_gb"]) == {"setup", "headline", "tp_decode", "tp_decode_70b"}, out["hbm_plan_gb"]
    assert out["hbm_peak_gb"] is None and "multi_timeout" not in out


def test_verdict_decoder_splits_every_bench_world():
    """bench.py's TP verdict at N = 4 / 8 needs a decoder whose heads split that many ways (an 8-rank
    rehearsal failed on tiny-dec's 4 heads before the choice depended on the world, then on
    tiny-dec-tp8's head dim 32)."""
    from docagents_amd.models.configs import decoder_config
    from docagents_amd.parallel.tp_verify import verdict_arch
    for w in (1, 2, 4, 8):
        c = decoder_config(verdict_arch(w))
        assert c.heads % w == 0 and c.kv_heads % w == 0 and c.ffn % (16 * w) == 0 and c.vocab % w == 0
        assert c.hidden // c.heads in (64, 96, 128)  # a head dim the GPU decode-attention kernels take


def test_bench_watchdog_ends_a_hung_block_with_the_json_line():
    """A multi-GPU block that never returns (a hung collective) must not cost the run its headline:
    past --block-budget-s every rank ends, rank 0 having printed the one JSON line with the blocks
    done so far and the block that hung; the launcher's status stays 0."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="2", DA_BENCH_HANG_BLOCK="tp_decode")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-rehearsal",
           "--enc", "tiny-enc", "--llm", "tiny-dec", "--batch", "2", "--steps", "1", "--warmup", "0",
           "--latency-reps", "1", "--ingest-docs", "0", "--index-rows", "2000", "--multi-iters", "2",
           "--breakdown", "0", "--max-new", "4", "--serving-requests", "4", "--block-budget-s", "3"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["value"] > 0 and out["multi_timeout"]["block"] == "tp_decode", out.get("multi_timeout")
    assert "rccl_search" in out and "serving_search" not in out
