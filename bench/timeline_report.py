"""Join a load run's request timeline (docagents_amd/utils/timeline.py, DA_REQ_TIMELINE=<dir>) into
where the concurrent cache-miss queries spent their time.

Per request (joined by question text): loadgen send -> query handler start (gateway + HTTP hops),
handler -> answer RPC sent (cache, embed_search, chunk tokens), answer RPC sent -> engine receipt,
receipt -> admission hand-off to the scheduler (held), admission -> reply (prefill + decode), reply
-> handler end -> loadgen receive. Plus the engine's decode-row occupancy over the ticks.

  python bench/timeline_report.py <dir> [--out report.json]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics


def load(d):
    ev = []
    for f in glob.glob(os.path.join(d, "*.jsonl")):
        with open(f) as fh:
            for ln in fh:
                try:
                    e = json.loads(ln)
                except ValueError:
                    continue
                e["src"] = os.path.basename(f).split(".")[0]
                ev.append(e)
    return sorted(ev, key=lambda e: e["t"])


def report(ev):
    per: dict = {}
    ticks = []
    by_text: dict = {}  # embed_search events carry the preprocessed question text
    for e in ev:
        if "t_text" in e:
            by_text.setdefault(e["t_text"], {}).setdefault(e["e"], e["t"])
    es = [r for r in by_text.values() if {"q_es_sent", "e_es_rx", "e_es_tx", "q_es_rx"} <= set(r)]
    for e in ev:
        k = e["e"]
        if k == "e_admit":
            for q in e["q"]:
                per.setdefault(q, {}).setdefault("e_admit", e["t"])
        elif k == "e_tick":
            ticks.append(e)
        elif "q" in e and e["q"] is not None:
            per.setdefault(e["q"], {}).setdefault(k, e["t"])
    segs = [("loadgen_to_gateway", "l_send", "g_rx"), ("gateway_to_query", "g_rx", "q_start"),
            ("gateway_in", "l_send", "q_start"), ("pre_answer", "q_start", "q_answer_sent"), ("search_stage", "q_start", "q_searched"),
            ("embed_cache_set", "q_searched", "q_embed_cached"), ("to_answer", "q_embed_cached", "q_answer_sent"),
            ("rpc_out", "q_answer_sent", "e_answer_rx"), ("held", "e_answer_rx", "e_admit"),
            ("in_engine", "e_admit", "e_answer_tx"), ("rpc_back", "e_answer_tx", "q_answer_rx"),
            ("post_answer", "q_answer_rx", "q_end"), ("query_to_gateway", "q_end", "g_tx"), ("gateway_to_loadgen", "g_tx", "l_recv"),
            ("gateway_out", "q_end", "l_recv"), ("total", "l_send", "l_recv")]
    out = {}
    full = [r for q, r in per.items() if "l_send" in r and "l_recv" in r
            and not q.startswith(("Serial question", "Warm-up question"))]
    for name, a, b in segs:
        xs = sorted((r[b] - r[a]) * 1000 for r in full if a in r and b in r)
        if xs:
            out[name] = {"n": len(xs), "mean_ms": round(statistics.mean(xs), 2), "p50_ms": round(xs[len(xs) // 2], 2),
                         "p99_ms": round(xs[min(len(xs) - 1, int(0.99 * len(xs)))], 2)}
    for name, a, b in (("es_rpc_in", "q_es_sent", "e_es_rx"), ("es_engine", "e_es_rx", "e_es_tx"),
                       ("es_rpc_back", "e_es_tx", "q_es_rx"), ("es_embed", "e_es_rx", "e_es_embedded"),
                       ("es_search", "e_es_embedded", "e_es_tx"), ("es_total", "q_es_sent", "q_es_rx"),
                       ("chunk_rows", "q_es_rx", "q_results")):
        xs = sorted((r[b] - r[a]) * 1000 for r in es)
        if xs:
            out[name] = {"n": len(xs), "mean_ms": round(statistics.mean(xs), 2), "p50_ms": round(xs[len(xs) // 2], 2),
                         "p99_ms": round(xs[min(len(xs) - 1, int(0.99 * len(xs)))], 2)}
    lags: dict = {}
    for e in ev:
        if e["e"] == "loop_lag":
            lags.setdefault(e["src"], []).append(e["ms"])
    if lags:
        out["loop_stalls"] = {src: {"n": len(x), "total_ms": round(sum(x), 1), "max_ms": max(x)}
                              for src, x in lags.items()}
    if full:
        t0 = min(r["l_send"] for r in full)
        t1 = max(r["l_recv"] for r in full)
        out["window_s"] = round(t1 - t0, 3)
        tk = [t for t in ticks if t0 <= t["t"] <= t1]
        if tk:
            w = sum(t["dt"] for t in tk)
            out["ticks"] = {"n": len(tk), "busy_s": round(w, 3),
                            "mean_active_rows_time_weighted": round(sum(t["n_active"] * t["dt"] for t in tk) / max(w, 1e-9), 1),
                            "admissions": sum(1 for t in tk if t["admitted"]),
                            "mean_admit_group": round(statistics.mean([t["admitted"] for t in tk if t["admitted"]] or [0]), 2),
                            "steps": sum(t["steps"] for t in tk)}
        # in-flight counts sampled every 50 ms: at loadgen, in the query handler, in the engine's rows
        samp = []
        t = t0
        while t < t1:
            lg = sum(1 for r in full if r["l_send"] <= t < r["l_recv"])
            qh = sum(1 for r in full if r.get("q_start", 1e30) <= t < r.get("q_end", -1))
            en = sum(1 for r in full if r.get("e_admit", 1e30) <= t < r.get("e_answer_tx", -1))
            samp.append((lg, qh, en))
            t += 0.05
        out["inflight_mean"] = {"loadgen": round(statistics.mean(s[0] for s in samp), 1),
                                "query_handler": round(statistics.mean(s[1] for s in samp), 1),
                                "engine_admitted": round(statistics.mean(s[2] for s in samp), 1)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    out = report(load(a.dir))
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
