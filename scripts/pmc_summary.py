"""Summarise rocprofv3 CSV output (kernel trace + separate FETCH_SIZE / WRITE_SIZE PMC passes)
into profiles/<tag>_pmc_summary.json, profiles/<tag>_kernel_stats.csv (rocprofv3 --stats: every
dispatch of the run, warm-up and copy-back runs included) and profiles/<tag>_kernel_stats_timed.csv
(the same statistics over the timed window only: the last_n tick launches before the skipped tail).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads exactly half of a
wide coalesced stream on gfx950, so hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024; the bulk kernel's
payload traffic is 16 B/lane coalesced, which is the calibrated case.
usage: python scripts/pmc_summary.py TAG KTRACE_DIR FETCH_DIR WRITE_DIR [last_n] [skip_tail]
(skip_tail: tick-kernel dispatches after the timed region, bench.py CONTROL_TIMING_STEPS)
"""
import csv
import glob
import json
import os
import shutil
import sys


def rows(d, pattern):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True)):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def short(name):
    for k in ("control_fastfb_kernel", "control_fast_kernel", "control_slow_kernel", "control_kernel",
              "bulk_small_kernel", "bulk_kernel", "bulk_meta_kernel", "tick_kernel", "bootstrap_kernel",
              "fill_slabs_kernel", "sum_committed_kernel", "traffic_kernel", "unpack_kernel", "pack_kernel",
              "plan_kernel", "scan_reduce_kernel", "scan_blocks_kernel", "scan_apply_kernel", "bounds_kernel",
              "apply_count_kernel", "apply_gather_kernel", "apply_total_kernel", "pool_kernel"):
        if k in name:
            return k
    return name[:60]


TICK_KERNELS = ("control_kernel", "control_fast_kernel", "control_fastfb_kernel", "control_slow_kernel",
                "bulk_kernel", "bulk_small_kernel", "pool_kernel")
# SKIP_HEAD=h (the bench's bring-up ticks + warm-up): the timed window is the last_n tick launches
# after the first h (more robust than counting the launches of the runs after the timed region)
HEAD = int(os.environ["SKIP_HEAD"]) if os.environ.get("SKIP_HEAD") else None


def window(k, xs, last_n, skip):
    """The last_n values before the skipped tail (tick kernels only), or after the first SKIP_HEAD."""
    if HEAD is not None and k in TICK_KERNELS:
        return xs[HEAD:HEAD + last_n]
    s = skip if k in TICK_KERNELS else 0
    return xs[max(len(xs) - last_n - s, 0):len(xs) - s]


def pmc(d, counter, last_n, skip=0):
    vals = {}
    for r in rows(d, "*counter_collection.csv"):
        if r.get("Counter_Name") != counter:
            continue
        k = short(r.get("Kernel_Name", ""))
        vals.setdefault(k, []).append((int(r.get("Dispatch_Id", 0)), float(r["Counter_Value"])))
    return {k: window(k, [v for _, v in sorted(x)], last_n, skip) for k, x in vals.items()}


def main():
    tag, kdir, fdir, wdir = sys.argv[1:5]
    last_n = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    skip = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.environ.get("PROFILES_DIR") or os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(kdir, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
    trace = rows(kdir, "*kernel_trace.csv")
    dur = {}
    for r in trace:
        k = short(r.get("Kernel_Name", ""))
        dur.setdefault(k, []).append((int(r.get("Dispatch_Id", 0)), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    with open(os.path.join(prof, f"{tag}_kernel_stats_timed.csv"), "w") as f:
        f.write("Name,Calls,AverageNs,MinNs,MaxNs,Window\n")
        for k in sorted(dur):
            d = window(k, [v for _, v in sorted(dur[k])], last_n, skip)
            if d:
                f.write(f"{k},{len(d)},{sum(d) / len(d):.1f},{min(d)},{max(d)},"
                        f"{'timed tick launches' if k in TICK_KERNELS else 'last dispatches'}\n")
    fetch = pmc(fdir, "FETCH_SIZE", last_n, skip)
    write = pmc(wdir, "WRITE_SIZE", last_n, skip)
    out = {"note": __doc__.strip().splitlines()[0], "last_n_dispatches": last_n, "skipped_tail": skip,
           "kernels": {}}
    for k in set(dur) | set(fetch):
        d = window(k, [v for _, v in sorted(dur.get(k, []))], last_n, skip)
        e = {"dispatches_averaged": len(d), "avg_duration_ns": sum(d) / len(d) if d else None}
        if k in fetch and k in write and fetch[k] and write[k]:
            fk = sum(fetch[k]) / len(fetch[k])
            wk = sum(write[k]) / len(write[k])
            e.update(fetch_size_kb=fk, write_size_kb=wk, hbm_bytes_per_launch=(2 * fk + wk) * 1024)
        out["kernels"][k] = e
    with open(os.path.join(prof, f"{tag}_pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
