"""SQ / LDS / MFMA counter passes (rocprofv3 --pmc, one pass per counter group, each on its own child run
of `bench.py --kernel-only`) for k_spread, k_interp, k_grid and the Nystrom setup's k_gemm_f64.

    python tools/pmc_sq.py --out profiles/r02_pmc_sq.csv [--n 1000000 --d 32 --nys 512]

Writes one CSV row per (kernel, counter): the mean value per dispatch.  Counter names are checked against
`rocprofv3 -L` first; unknown ones are dropped (and listed) instead of failing the pass.
"""
import argparse
import csv
import re
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [
    ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY",
     "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_WAVES"],
    ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
     "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"],
    ["SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_INSTS_VALU_MFMA_F64", "SQ_ACTIVE_INST_LDS",
     "SQ_INST_CYCLES_VMEM", "SQ_ACTIVE_INST_MISC", "GRBM_GUI_ACTIVE", "GRBM_COUNT"],
]
KERNELS = {"k_spread": "k_spread", "k_interp": "k_interp", "k_grid": "k_grid", "k_gemm_f64": "k_gemm_f64"}


def available():
    r = subprocess.run(["rocprofv3", "-L"], capture_output=True, text=True, timeout=120, cwd="/tmp")
    names = set()
    for line in (r.stdout + r.stderr).splitlines():
        for tok in line.replace(",", " ").replace(":", " ").split():
            if tok.startswith(("SQ_", "GRBM_", "TCC_", "TCP_")):
                names.add(tok)
    return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--nys", type=int, default=512)
    args = ap.parse_args()
    have = available()
    rows, dropped = [], []
    env = dict(os.environ, TMPDIR="/tmp")
    for i, counters in enumerate(PASSES):
        use = [c for c in counters if c in have] if have else counters
        dropped += [c for c in counters if c not in use]
        if not use:
            continue
        d_out = os.path.join(ROOT, "gpurun_out", "pmc_sq", f"pass{i}")
        shutil.rmtree(d_out, ignore_errors=True)
        cmd = ["rocprofv3", "--pmc", *use, "--output-format", "csv", "-d", d_out, "-o", "pmc", "--",
               sys.executable, os.path.join(ROOT, "bench.py"), "--kernel-only", "--n", str(args.n), "--d",
               str(args.d), "--kernel-only-nys", str(args.nys)]
        r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(f"pass {i} failed rc={r.returncode}: {r.stderr[-2000:]}", file=sys.stderr)
            sys.exit(1)
        path = None
        for root, _, files in os.walk(d_out):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    path = os.path.join(root, f)
        sums = {}
        with open(path) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"]
                key = next((k for k in KERNELS if k in name), None)
                if key is None:
                    continue
                # template instances: keep the variant in the key (interp plain / grad / dot)
                m = re.search(r"(k_\w+(?:<[^()]*>)?)", name)
                variant = m.group(1) if m else key
                s = sums.setdefault((variant, row["Counter_Name"]), {})
                s.setdefault(row.get("Dispatch_Id", len(s)), 0.0)
                s[row.get("Dispatch_Id", len(s))] += float(row["Counter_Value"])
        for (variant, counter), per in sorted(sums.items()):
            rows.append({"kernel": variant, "counter": counter, "dispatches": len(per),
                         "mean_per_dispatch": sum(per.values()) / len(per)})
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["kernel", "counter", "dispatches", "mean_per_dispatch"])
        w.writeheader()
        w.writerows(rows)
    print(f"wrote {args.out}: {len(rows)} rows; dropped (not in rocprofv3 -L): {dropped}")


if __name__ == "__main__":
    main()
