"""Summarize a profiles/collect.sh run (gpurun_out/prof_<tag>/) into profiles/<tag>_summary.md
and merge per-kernel HBM traffic into profiles/traffic.json (read by bench.py).

    python profiles/summarize.py <tag> [--config c2]

HBM traffic per launch follows MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7:
FETCH_SIZE and WRITE_SIZE come from separate --pmc passes, are in KiB, and on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) streaming read, so
    traffic_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
The x2 is calibrated for coalesced 16 B/lane streams (rs_apply_kernel) and for the SHA kernel's
per-lane loads (one 1 MiB-apart stream per lane): tools/ubench_fetch.hip reads a known byte count
in each pattern and FETCH_SIZE reports exactly half (profiles/r1y_fetch_calibration.log).
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    for k in ("rs_apply_var_kernel", "rs_apply_kernel", "rs_encode_bs_kernel", "sha256_lane_kernel", "sha256_split_kernel", "fill_kernel",
              "encode_hash_kernel", "copyBuffer"):
        if k in name:
            return k
    return name[:40]


LAUNCHES = None  # (a, b): per kernel, only its launches a..b-1 in dispatch order (--launches a:b)


def pmc(path):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    if not os.path.exists(path):
        return out, dur
    seen = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        i = seen[(k, r["Counter_Name"])]
        seen[(k, r["Counter_Name"])] += 1
        if LAUNCHES and k in ("rs_apply_var_kernel",) and not LAUNCHES[0] <= i < LAUNCHES[1]:
            continue
        out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return out, dur


def mean(v):
    return sum(v) / len(v) if v else float("nan")


def main():
    global LAUNCHES
    tag = sys.argv[1]
    if "--launches" in sys.argv:  # c3e2: the reconstruct_data launches come first
        a, b = sys.argv[sys.argv.index("--launches") + 1].split(":")
        LAUNCHES = (int(a), int(b))
    config = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "c2"
    # FETCH_SIZE multiplier: 2 for 16 B/lane streaming reads (the guide's gfx950 calibration);
    # 1 for the RS(20,p) fused build's 8 B/lane reads, whose two 64-B halves of a line are read
    # one ~5 us step apart: calibrated independently by tools/ubench_fetch.hip's wide8_steps
    # kernel, which reads a known 21.47 GB in that exact pattern and pacing and gets FETCH_SIZE =
    # 1.000 x the bytes (profiles/r2_fetch_calibration.log; unpaced the halves merge: 1.78).
    fmult = float(sys.argv[sys.argv.index("--fetch-mult") + 1]) if "--fetch-mult" in sys.argv \
        else 2.0
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    sq, _ = pmc(os.path.join(src, "pmc_sq", "run_counter_collection.csv"))
    fetch, _ = pmc(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write, _ = pmc(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    lines = [f"# rocprofv3 summary `{tag}` ({config})", "",
             "Source: `profiles/collect.sh` on one MI355X (gfx950); raw CSVs under "
             f"`profiles/{tag}/`.", "",
             "## Kernel trace (`--kernel-trace --stats`)", "",
             "| kernel | calls | avg ms | min ms | max ms |", "|---|---|---|---|---|"]
    for r in stats:
        lines.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs'])/1e6:.3f} | "
                     f"{float(r['MinNs'])/1e6:.3f} | {float(r['MaxNs'])/1e6:.3f} |")
    lines += ["", "## Counters (separate `--pmc` passes; per-launch means)", ""]
    if LAUNCHES:
        lines += [f"rs_apply_var_kernel: launches {LAUNCHES[0]}..{LAUNCHES[1] - 1} only (the "
                  "reconstruct_data steps; the reconstruct launches timed beside them follow).", ""]
    lines += [
              "| kernel | clock GHz (GRBM_GUI_ACTIVE/8/dur) | SQ_WAVES | VALU insts/wave | "
              f"FETCH_SIZE KiB | WRITE_SIZE KiB | HBM traffic GB ({fmult:g}xFETCH+WRITE) |",
              "|---|---|---|---|---|---|---|"]
    traffic = {}
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):
        traffic = json.load(open(tpath))
    for k in sq:
        if k in ("copyBuffer",):
            continue
        c = sq[k]
        _, durs = pmc(os.path.join(src, "pmc_sq", "run_counter_collection.csv"))
        d_ms = mean(durs[k])
        ghz = mean(c["GRBM_GUI_ACTIVE"]) / 8 / (d_ms / 1e3) / 1e9 if d_ms else float("nan")
        waves = mean(c["SQ_WAVES"])
        vpw = mean(c["SQ_INSTS_VALU"]) / waves if waves else float("nan")
        f = mean(fetch[k].get("FETCH_SIZE", []))
        w = mean(write[k].get("WRITE_SIZE", []))
        tb = (fmult * f + w) * 1024 if f == f and w == w else None
        lines.append(f"| {k} | {ghz:.2f} | {waves:.0f} | {vpw:.0f} | {f:.0f} | {w:.0f} | "
                     f"{tb/1e9 if tb else float('nan'):.2f} |")
        if tb and k in ("rs_apply_kernel", "rs_apply_var_kernel", "sha256_lane_kernel",
                        "encode_hash_kernel", "rs_encode_bs_kernel"):
            traffic.setdefault(config, {})[k] = {
                "bytes_per_launch": int(tb),
                "fetch_kib": f, "write_kib": w,
                # x2 measured for both read patterns (tools/ubench_fetch.hip,
                # profiles/r1y_fetch_calibration.log): coalesced 16 B/lane and per-lane streams
                "calibrated": k in ("rs_apply_kernel", "rs_apply_var_kernel", "encode_hash_kernel",
                                    "sha256_lane_kernel", "rs_encode_bs_kernel") or fmult != 2.0,
                "fetch_mult": fmult,
                "source": f"profiles/{tag}_summary.md",
            }
    with open(os.path.join(ROOT, "profiles", f"{tag}_summary.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    with open(tpath, "w") as fh:
        json.dump(traffic, fh, indent=1)
    # keep the raw CSVs that the summary is built from
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for sub in ("trace", "pmc_sq", "pmc_fetch", "pmc_write"):
        for fn in ("run_kernel_stats.csv", "run_counter_collection.csv"):
            p = os.path.join(src, sub, fn)
            if os.path.exists(p):
                with open(p) as fi, open(os.path.join(dst, f"{sub}_{fn}"), "w") as fo:
                    fo.write(fi.read())
    print("\n".join(lines))


if __name__ == "__main__":
    main()
