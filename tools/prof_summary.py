"""Per-kernel durations from a rocprofv3 kernel trace of `bench.py` (TEST/EVIDENCE tooling).

    python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps K --out profiles/rNN_x.json

The bench's timed region is its last matvec loops: K uninstrumented steps, then K steps with
dispatch-attached events (bench.py).  This reports, per kernel of the matvec, the mean duration over all
dispatches of the run and over the last 2K of them (those two loops), and the whole-matvec span
(first spread start to last interp end of the last 2K matvecs / 2K).  The bench line's roofline
(achieved = 8n(d+1) / avg_launch_ms) can be recomputed from the `timed_mean_ms` here.
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=32)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    kinds = {"spread": "k_spread<", "grid": "k_grid(", "interp": "k_interp<false, 1024, false"}
    out = {"trace": args.trace, "steps": args.steps, "kernels": {}}
    for key, pat in kinds.items():
        durs = [(e - s) * 1e-6 for s, e, name in rows if pat in name]
        if not durs:
            continue
        last = durs[-2 * args.steps:]
        out["kernels"][key] = {"dispatches": len(durs), "all_mean_ms": sum(durs) / len(durs),
                               "timed_dispatches": len(last), "timed_mean_ms": sum(last) / len(last)}
    sp = [(s, e) for s, e, name in rows if kinds["spread"] in name][-2 * args.steps:]
    ip = [(s, e) for s, e, name in rows if kinds["interp"] in name][-2 * args.steps:]
    if sp and ip:
        out["matvec_span_ms_timed"] = (ip[-1][1] - sp[0][0]) * 1e-6 / len(sp)
    sp_ms = out["kernels"].get("spread", {}).get("timed_mean_ms")
    if sp_ms:
        b = 8 * args.n * (args.d + 1)
        out["spread_frac_survey_bytes"] = b / (sp_ms * 1e-3) / 8e12
        out["spread_survey_bytes"] = b
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
