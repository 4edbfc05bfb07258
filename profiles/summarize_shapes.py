"""Summarize a profiles/collect.sh run of a command that launches one kernel at several shapes
(the default bench line: the C2 headline, the north_star block's full-size encode and 2-erasure
reconstruct_data, and the end-to-end forms' 256-part batches) into profiles/<tag>_summary.md,
one row per (kernel, grid size), and merge the full-size launch of each kernel (its largest grid)
into profiles/traffic.json under --config (read by bench.py).

    python profiles/summarize_shapes.py <tag> [--config c2] [--fetch-mult 2]
                                        [--grid encode_hash_kernel=131072,...] [--committed]

--committed re-reads the CSVs already copied to profiles/<tag>/ (no GPU run needed).

--grid names the launch shape to merge for a kernel when its largest grid is not the config's
(the default line also runs BASELINE's C3 / C4 configurations: C4's fused kernel and C3's
reconstruct have larger grids than the C2 launches the c2 entries describe).

Durations come from the kernel trace (run_kernel_trace.csv, every dispatch); counters from the
separate --pmc passes, matched to the same (kernel, grid).  HBM traffic per launch, as
profiles/summarize.py: 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 (gfx950 FETCH_SIZE reports half
the bytes of these streaming reads, tools/ubench_fetch.hip).

VALU utilisation per launch, from the SQ pass (units stated in the table): GRBM_GUI_ACTIVE counts
cycles summed over the 8 XCDs, so the launch lasts GRBM_GUI_ACTIVE / 8 cycles and offers
(GRBM_GUI_ACTIVE / 8) x 1024 SIMD-cycles (256 CUs x 4 SIMDs); SQ_INSTS_VALU counts wave64 VALU
instructions.  SIMD-cycles per VALU instruction = that ratio; a SIMD issues at most one VALU
wave-instruction per 4 cycles to one wave (the lone-wave issue floor, MI355X_MICROARCH.md), so
"VALU busy" = 4 x SQ_INSTS_VALU / SIMD-cycles.  SQ_ACTIVE_INST_VALU equals SQ_INSTS_VALU on gfx950
(one count per instruction), so it adds no separate figure.  The full-size launch of each kernel
goes into profiles/valu.json under --config (read by bench.py's valu_roofline).
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize import short  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRAFFIC_KERNELS = ("rs_apply_kernel", "rs_apply_var_kernel", "sha256_lane_kernel",
                   "encode_hash_kernel", "rs_encode_bs_kernel")


def mean(v):
    return sum(v) / len(v) if v else float("nan")


def trace_groups(path):
    """(kernel, grid) -> list of durations in ms, from run_kernel_trace.csv."""
    g = collections.defaultdict(list)
    if not os.path.exists(path):
        return g
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        grid = int(r["Grid_Size"]) if "Grid_Size" in r else \
            int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        g[(k, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return g


def pmc_groups(path):
    """(kernel, grid) -> counter -> list of per-launch values; and -> list of durations."""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    if not os.path.exists(path):
        return out, dur
    for r in csv.DictReader(open(path)):
        key = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
        out[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return out, dur


def main():
    tag = sys.argv[1]
    config = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "c2"
    fmult = float(sys.argv[sys.argv.index("--fetch-mult") + 1]) if "--fetch-mult" in sys.argv \
        else 2.0
    pick = {}
    if "--grid" in sys.argv:
        for kv in sys.argv[sys.argv.index("--grid") + 1].split(","):
            k, g = kv.split("=")
            pick[k] = int(g)
    committed = "--committed" in sys.argv
    src = os.path.join(ROOT, "profiles", tag) if committed else \
        os.path.join(ROOT, "gpurun_out", f"prof_{tag}")

    def csv_path(sub, fn):  # gpurun_out/prof_<tag>/<sub>/<fn>, or its committed copy
        return os.path.join(src, f"{sub}_{fn}") if committed else os.path.join(src, sub, fn)
    tr = trace_groups(csv_path("trace", "run_kernel_trace.csv"))
    sq, sq_dur = pmc_groups(csv_path("pmc_sq", "run_counter_collection.csv"))
    fetch, _ = pmc_groups(csv_path("pmc_fetch", "run_counter_collection.csv"))
    write, _ = pmc_groups(csv_path("pmc_write", "run_counter_collection.csv"))
    cmd = open(os.path.join(src, "command.txt")).read().strip() \
        if os.path.exists(os.path.join(src, "command.txt")) else "bench.py"
    lines = [f"# rocprofv3 summary `{tag}` ({config})", "",
             f"Command: `{cmd}` on one MI355X (gfx950), profiled by `profiles/collect.sh`; raw "
             f"CSVs under `profiles/{tag}/`.  One row per kernel and grid size: the same kernel "
             "runs at the full C2 shape, at the end-to-end forms' 256-part batches and (the default "
             "line) at BASELINE's C3 / C4 shapes.", "",
             "## Kernel trace (`--kernel-trace --stats`), per dispatch shape", "",
             "| kernel | grid (work-items) | calls | avg ms | min ms | max ms |",
             "|---|---|---|---|---|---|"]
    for (k, grid), durs in sorted(tr.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| {k} | {grid} | {len(durs)} | {mean(durs):.3f} | {min(durs):.3f} | "
                     f"{max(durs):.3f} |")
    lines += ["", "## Counters (separate `--pmc` passes; per-launch means over the launches of "
              "that shape)", "",
              "| kernel | grid | clock GHz (GRBM_GUI_ACTIVE/8/dur) | SQ_WAVES | VALU insts/wave | "
              "SIMD-cycles per VALU inst ((GRBM_GUI_ACTIVE/8)x1024/SQ_INSTS_VALU) | "
              "VALU busy (4xSQ_INSTS_VALU/SIMD-cycles) | "
              f"FETCH_SIZE KiB | WRITE_SIZE KiB | HBM traffic GB ({fmult:g}xFETCH+WRITE) |",
              "|---|---|---|---|---|---|---|---|---|---|"]
    valu_table = {}
    vpath = os.path.join(ROOT, "profiles", "valu.json")
    if os.path.exists(vpath):
        valu_table = json.load(open(vpath))
    valu_big = {}
    traffic = {}
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):
        traffic = json.load(open(tpath))
    biggest = {}
    for key in sorted(sq, key=lambda kk: (kk[0], -kk[1])):
        k, grid = key
        if k in ("copyBuffer",):
            continue
        c = sq[key]
        d_ms = mean(sq_dur[key])
        ghz = mean(c["GRBM_GUI_ACTIVE"]) / 8 / (d_ms / 1e3) / 1e9 if d_ms else float("nan")
        waves = mean(c["SQ_WAVES"])
        vpw = mean(c["SQ_INSTS_VALU"]) / waves if waves else float("nan")
        simd_cycles = mean(c["GRBM_GUI_ACTIVE"]) / 8 * 1024
        insts = mean(c["SQ_INSTS_VALU"])
        cpi = simd_cycles / insts if insts else float("nan")
        busy = 4 * insts / simd_cycles if simd_cycles else float("nan")
        f = mean(fetch[key].get("FETCH_SIZE", []))
        w = mean(write[key].get("WRITE_SIZE", []))
        tb = (fmult * f + w) * 1024 if f == f and w == w else None
        lines.append(f"| {k} | {grid} | {ghz:.2f} | {waves:.0f} | {vpw:.0f} | {cpi:.2f} | "
                     f"{busy:.3f} | {f:.0f} | {w:.0f} | {tb / 1e9 if tb else float('nan'):.2f} |")
        vchosen = grid == pick[k] if k in pick else grid > valu_big.get(k, (0, None))[0]
        if insts and k in TRAFFIC_KERNELS and vchosen:
            valu_big[k] = (grid, {"simd_cycles_per_valu": round(cpi, 3), "valu_busy": round(busy, 4),
                                  "valu_insts": insts, "simd_cycles": simd_cycles, "grid": grid,
                                  "source": f"profiles/{tag}_summary.md"})
        chosen = grid == pick[k] if k in pick else grid > biggest.get(k, (0, None))[0]
        if tb and k in TRAFFIC_KERNELS and chosen:
            biggest[k] = (grid, {"bytes_per_launch": int(tb), "fetch_kib": f, "write_kib": w,
                                 "grid": grid, "calibrated": True, "fetch_mult": fmult,
                                 "source": f"profiles/{tag}_summary.md"})
    for k, (_, entry) in biggest.items():
        traffic.setdefault(config, {})[k] = entry
    for k, (_, entry) in valu_big.items():
        valu_table.setdefault(config, {})[k] = entry
    with open(vpath, "w") as fh:
        json.dump(valu_table, fh, indent=1)
    with open(os.path.join(ROOT, "profiles", f"{tag}_summary.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    with open(tpath, "w") as fh:
        json.dump(traffic, fh, indent=1)
    dst = os.path.join(ROOT, "profiles", tag)
    if committed:  # the CSVs are already there
        print("\n".join(lines))
        return
    os.makedirs(dst, exist_ok=True)
    for sub in ("trace", "pmc_sq", "pmc_fetch", "pmc_write"):
        for fn in ("run_kernel_stats.csv", "run_counter_collection.csv", "run_kernel_trace.csv"):
            p = os.path.join(src, sub, fn)
            if os.path.exists(p):
                with open(p) as fi, open(os.path.join(dst, f"{sub}_{fn}"), "w") as fo:
                    fo.write(fi.read())
    for fn in ("trace_bench.log", "command.txt"):
        p = os.path.join(src, fn)
        if os.path.exists(p):
            with open(p) as fi, open(os.path.join(dst, fn), "w") as fo:
                fo.write(fi.read())
    print("\n".join(lines))


if __name__ == "__main__":
    main()
