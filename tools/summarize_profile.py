#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (rocprofv3 CSVs under gpurun_out/prof_<tag>) into
profiles/<tag>/: kernel_stats.csv (copied), summary.json and summary.md.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB
(x1024); on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled;
FETCH and WRITE come from separate --pmc passes.
"""
import csv
import collections
import json
import os
import shutil
import sys

STEP_KERNELS = None


def short(name):
    n = name.split("(")[0]
    for k, tag in (("actor_chain_kernel", "actor_chain"), ("critic_chain_kernel", "critic_loss_chain"),
                   ("chain_fwd_kernel", "chain_fwd"), ("adam_net_kernel", "sac_adam"),
                   ("gemm_jobs", "sac_wgrad")):
        if k in n:
            return tag
    if "reduce_adam_kernel" in n:
        return "reduce_adam"
    if "fc_bwd_kernel" in n:
        return "FcBwd"
    if "wgrad23_kernel" in n:
        return "Wgrad23"
    if "lnc3_conv12_bwd" in n:
        return "LnConv12Bwd"
    if "fwd_chain_kernel" in n:
        return "FwdChain"
    if "conv1_fwd_s2d" in n:
        return "Conv1Fwd"
    if "conv12_bwd_s2d" in n:
        return "Conv12Bwd"
    if "conv12_fwd_s2d" in n:
        return "Conv12Fwd"
    if "lnc3_bwd" in n:
        return "LnConv3Bwd"
    if "head_step" in n:
        return "head_step"
    if "gemm_tile" in n or "gemm_wg" in n or "gemm_rc" in n:
        for tag in ("Conv3LnFwd", "FcHeadsFwd"):
            if tag in n:
                return tag
    for tag in ("Conv1Fwd", "Conv2Fwd", "Conv3Fwd", "FcFwd", "HeadsFwd", "HeadsDgrad", "FcDgrad",
                "Conv3Dgrad", "Conv2Dgrad", "HeadsWgrad", "FcWgrad", "Conv3Wgrad", "Conv2Wgrad",
                "Conv1Wgrad", "ln_fwd", "ln_bwd", "loss_head", "reduce_grads", "adam", "sumsq",
                "pack_params", "conv_fwd", "conv_dgrad", "conv_wgrad", "fused"):
        if tag in n:
            return tag
    return n[:60]


def main(tag, src_root="gpurun_out", dst_root="profiles"):
    src = os.path.join(src_root, f"prof_{tag}")
    dst = os.path.join(dst_root, tag)
    os.makedirs(dst, exist_ok=True)
    stats = list(csv.DictReader(open(os.path.join(src, "stats", "run_kernel_stats.csv"))))
    shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub, cname in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == cname:
                ctr[r["Kernel_Name"]][cname].append(float(r["Counter_Value"]))
    # per-launch durations from the kernel trace: the median and the mean of the second half of
    # the launches (the run's first launches run at a lower clock: ~77 vs ~71 us for the fused
    # backward in r04zc, so the all-launch mean sits above the bench's steady-state timing)
    durs = collections.defaultdict(list)
    tp = os.path.join(src, "stats", "run_kernel_trace.csv")
    if os.path.exists(tp):
        for r in csv.DictReader(open(tp)):
            durs[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = []
    total_ns = sum(float(r["TotalDurationNs"]) for r in stats)
    for r in stats:
        name = r["Name"]
        c = ctr.get(name, {})
        fetch = c.get("FETCH_SIZE")
        write = c.get("WRITE_SIZE")
        fb = 2 * 1024 * sum(fetch) / len(fetch) if fetch else None
        wb = 1024 * sum(write) / len(write) if write else None
        dd = durs.get(name, [])
        med = sorted(dd)[len(dd) // 2] if dd else None
        late = sum(dd[len(dd) // 2:]) / len(dd[len(dd) // 2:]) if dd else None
        out.append({"kernel": short(name), "name": name[:200], "calls": int(r["Calls"]),
                    "avg_us": float(r["AverageNs"]) / 1e3, "median_us": med, "late_half_avg_us": late,
                    "pct": float(r["Percentage"]),
                    "hbm_read_bytes": fb, "hbm_write_bytes": wb,
                    "hbm_bytes": (fb or 0) + (wb or 0) if (fb is not None or wb is not None) else None})
    for k in ("bench_stats.json",):
        p = os.path.join(src, k)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, k))
    dtype, algo = "bf16", "impala"
    bj = os.path.join(src, "bench_stats.json")
    if os.path.exists(bj):
        try:
            line = json.loads(open(bj).read().strip().splitlines()[-1])
            dtype = line.get("dtype", "bf16")
            algo = line.get("algo") or ("ppo" if "PPO" in line.get("metric", "") else
                                        "sac" if "SAC" in line.get("metric", "") else "impala")
        except Exception:
            pass
    import datetime
    created = datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
    json.dump({"tag": tag, "algo": algo, "dtype": dtype, "created": created,
               "total_kernel_ns": total_ns, "kernels": out},
              open(os.path.join(dst, "summary.json"), "w"), indent=1)
    with open(os.path.join(dst, "summary.md"), "w") as f:
        f.write(f"# rocprofv3 summary `{tag}`\n\n`tools/profile.sh {tag}` = `rocprofv3 --kernel-trace --stats` "
                "over `bench.py --steps 20 --warmup 20` (r04zc and earlier: `--warmup 3`; every launch of the run: warmup, kernel selection, the "
                "timed and the stamped steps), then separate `--pmc FETCH_SIZE` "
                "and `--pmc WRITE_SIZE` passes. HBM bytes per launch: FETCH_SIZE×1024×2 (gfx950 half-count "
                "correction) + WRITE_SIZE×1024. Median and second-half mean per launch from the kernel "
                "trace (the first launches of a run are clocked lower).\n\n")
        f.write("| kernel | calls | avg µs | median µs | 2nd-half avg µs | % time | HBM read MB | HBM write MB |\n"
                "|---|---|---|---|---|---|---|---|\n")
        for o in out:
            rd = f"{o['hbm_read_bytes'] / 1e6:.2f}" if o["hbm_read_bytes"] is not None else "-"
            wr = f"{o['hbm_write_bytes'] / 1e6:.2f}" if o["hbm_write_bytes"] is not None else "-"
            md = f"{o['median_us']:.2f}" if o["median_us"] is not None else "-"
            lt = f"{o['late_half_avg_us']:.2f}" if o["late_half_avg_us"] is not None else "-"
            f.write(f"| {o['kernel']} | {o['calls']} | {o['avg_us']:.2f} | {md} | {lt} | {o['pct']:.2f} | {rd} | {wr} |\n")
    print(open(os.path.join(dst, "summary.md")).read())


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
