"""Summarise a tools/profile.sh output directory into one JSON for profiles/.

Per kernel (matched by a name prefix): dispatches, average duration from the kernel trace, and
per-dispatch averages of FETCH_SIZE / WRITE_SIZE / SQ_INSTS_* from the separate --pmc passes.
HBM bytes follow MI355X_MICROARCH.md §HBM: rocprofv3 reports FETCH_SIZE and WRITE_SIZE in KiB.

Read-scale rule (one rule for every summary, round 3 on): on gfx950 FETCH_SIZE counts exactly
half the bytes of a wide (16 B/lane) coalesced streaming read (global_load and LDS-DMA alike);
other access widths are uncalibrated. So a kernel whose reads are all 16-B/lane streams -- the
dense chains (chain_block, chain_block64, chain_dense, chain_split: LDS-DMA rows) and the folds -- gets
2 x FETCH_SIZE; every other kernel (the CSR chains: 4-B/lane entry loads and scattered 4/8-B
gathers) gets FETCH_SIZE as counted (1 x), i.e. its gathers at the fabric-request granularity the
counter reports. --read-scale overrides the rule for every kernel.

usage: python tools/pmc_summary.py <prof dir> <out.json> [--workload NAME]
"""
import argparse
import csv
import json
import os
import statistics

KERNELS = ("psgd::chain_block64", "psgd::chain_block", "psgd::chain_sparse_spec", "psgd::chain_sparse_lds", "psgd::chain_sparse",
           "psgd::chain_dense", "psgd::chain_split", "psgd::chain_general", "psgd::fold_kernel", "psgd::fold_f32_kernel",
           "psgd::fold_scaled_kernel", "psgd::wf32_init_kernel", "psgd::w64_init_kernel", "psgd::margin_loss_kernel",
           "psgd::logistic_loss64_kernel")


STREAM_KERNELS = ("psgd::chain_block", "psgd::chain_dense", "psgd::chain_split", "psgd::fold_kernel", "psgd::fold_f32_kernel",
                  "psgd::fold_scaled_kernel", "psgd::wf32_init_kernel")


def read_scale(kernel):
    """2 for kernels whose reads are all 16-B/lane coalesced streams, else 1 (see above)."""
    return 2.0 if kernel.startswith(STREAM_KERNELS) else 1.0


def short(name):
    for k in KERNELS:
        if k in name:
            return name[name.index(k):].split("(")[0]
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof")
    ap.add_argument("out")
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--rows", type=int, default=0, help="rows one chain launch processed")
    ap.add_argument("--read-scale", type=float, default=0.0,
                    help="bytes per FETCH_SIZE byte for every kernel (default 0: the per-kernel rule above)")
    a = ap.parse_args()
    out = {"workload": a.workload, "source": "rocprofv3 (tools/profile_round.sh)", "kernels": {},
           "fetch_size_scale": a.read_scale or "per kernel: 2 for 16-B/lane streams (dense chains, folds), "
                                                "1 otherwise (tools/pmc_summary.py)"}
    if a.rows:
        out["rows_per_launch"] = a.rows
    trace = os.path.join(a.prof, "trace", "run_kernel_trace.csv")
    if os.path.exists(trace):
        for r in csv.DictReader(open(trace)):
            k = short(r["Kernel_Name"])
            if not k:
                continue
            e = out["kernels"].setdefault(k, {"durations_ns": []})
            e["durations_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for sub in ("fetch", "write", "insts"):
        path = os.path.join(a.prof, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            if not k:
                continue
            e = out["kernels"].setdefault(k, {"durations_ns": []})
            e.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, e in out["kernels"].items():
        d = e.pop("durations_ns")
        if d:
            e["dispatches"] = len(d)
            e["avg_duration_ms"] = statistics.mean(d) / 1e6
        for c in list(e):
            if isinstance(e[c], list):
                e[c] = statistics.mean(e[c])
        if "FETCH_SIZE" in e:
            scale = a.read_scale or read_scale(k)
            e["fetch_size_scale"] = scale
            e["hbm_read_bytes"] = scale * e["FETCH_SIZE"] * 1024   # KiB -> B (+ gfx950 correction)
        if "WRITE_SIZE" in e:
            e["hbm_write_bytes"] = e["WRITE_SIZE"] * 1024
        if "hbm_read_bytes" in e:
            e["hbm_bytes"] = e["hbm_read_bytes"] + e.get("hbm_write_bytes", 0.0)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
