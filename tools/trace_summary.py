"""Markdown summary of a rocprofv3 kernel trace of the default bench command (tools/r6_check.sh):
the launches the bench line times, by workgroup count, against the line's own HIP-event figures,
and the top kernels by total time.
    python3 tools/trace_summary.py <trace dir> <bench log> [<stats csv as committed>] \
        > profiles/r6/final/c2_trace_summary.md"""
import collections
import csv
import json
import os
import sys


def main(trace_dir, bench_log, stats=None):
    stats = stats or os.path.join(trace_dir, "run_kernel_stats.csv")
    rows = list(csv.DictReader(open(os.path.join(trace_dir, "run_kernel_trace.csv"))))
    line = json.loads([x for x in open(bench_log) if x.startswith("{")][-1])
    groups = collections.defaultdict(list)
    for r in rows:
        wg = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
        name = r["Kernel_Name"].replace("cec::(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0]
        groups[(name, wg)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    ns, bc = line["north_star"], line["baseline_configs"]
    want = [("C2 headline", "encode_hash_kernel<4, 256, 0, 10, 4, false, false>", line["ms_per_step"]),
            ("north_star encode", "rs_encode_bs_kernel<10, 4>", ns["encode"]["ms"]),
            ("north_star 2-erasure reconstruct_data", "rs_apply_var_kernel<true, 4, 2, true, 2, 10, 5>",
             ns["reconstruct_data_2_erasures"]["ms"]),
            ("C4 RS(20,8) encode + SHA-256", "encode_hash_kernel<8, 64, 0, 20, 8, true, true>",
             bc["c4_encode_hash"]["ms"]),
            ("C3 1-4 erasures", "rs_apply_var_kernel<true, 4, 2, true, 4, 10, 5>", bc["c3_reconstruct"]["ms"])]
    print("# Round 6: kernel trace of the default command on the final tree\n")
    print("`rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py --steps 10 "
          "--warmup 3 --no-cpu-baseline` (`tools/r6_check.sh`; raw stats: "
          f"`{stats}`; this file: `tools/trace_summary.py`).  Trace only: "
          "no hot-path kernel changed in rounds 5-6, so the PMC passes (HBM traffic, SQ counters) "
          "of `profiles/r4e_c2_summary.md` still describe them; this run checks that the round-6 "
          "tree's launches take what the bench line's HIP events say.\n")
    print("| launch | kernel (workgroups) | calls | rocprof avg ms | bench line (HIP events) ms |")
    print("|---|---|---|---|---|")
    for label, kern, ms in want:
        best = max(((k, v) for k, v in groups.items() if k[0] == kern), key=lambda kv: sum(kv[1]),
                   default=None)
        if best is None:
            continue
        (name, wg), ds = best
        print(f"| {label} | `{name}` ({wg}) | {len(ds)} | {sum(ds) / len(ds):.3f} | {ms:.3f} |")
    print(f"\nBench line of this run: value {line['value']} GB/s, ms_per_step {line['ms_per_step']}, "
          f"north_star {ns['encode']['frac']} / {ns['reconstruct_data_2_erasures']['frac']}.\n")
    print("Top kernels by total time:\n")
    print("| kernel | workgroups | calls | avg ms |")
    print("|---|---|---|---|")
    top = sorted(groups.items(), key=lambda kv: -sum(kv[1]))[:12]
    for (name, wg), ds in top:
        print(f"| `{name[:70]}` | {wg} | {len(ds)} | {sum(ds) / len(ds):.3f} |")


if __name__ == "__main__":
    main(*sys.argv[1:4])
