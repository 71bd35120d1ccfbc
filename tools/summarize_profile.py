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
    out = []
    total_ns = sum(float(r["TotalDurationNs"]) for r in stats)
    for r in stats:
        name = r["Name"]
        c = ctr.get(name, {})
        fetch = c.get("FETCH_SIZE")
        write = c.get("WRITE_SIZE")
        fb = 2 * 1024 * sum(fetch) / len(fetch) if fetch else None
        wb = 1024 * sum(write) / len(write) if write else None
        out.append({"kernel": short(name), "name": name[:200], "calls": int(r["Calls"]),
                    "avg_us": float(r["AverageNs"]) / 1e3, "pct": float(r["Percentage"]),
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
    json.dump({"tag": tag, "algo": algo, "dtype": dtype, "total_kernel_ns": total_ns, "kernels": out},
              open(os.path.join(dst, "summary.json"), "w"), indent=1)
    with open(os.path.join(dst, "summary.md"), "w") as f:
        f.write(f"# rocprofv3 summary `{tag}`\n\n`tools/profile.sh {tag}` = `rocprofv3 --kernel-trace --stats` "
                "over `bench.py --steps 20 --warmup 3` (every launch of the run: warmup, kernel selection, the "
                "timed and the stamped steps), then separate `--pmc FETCH_SIZE` "
                "and `--pmc WRITE_SIZE` passes. HBM bytes per launch: FETCH_SIZE×1024×2 (gfx950 half-count "
                "correction) + WRITE_SIZE×1024.\n\n")
        f.write("| kernel | calls | avg µs | % time | HBM read MB | HBM write MB |\n|---|---|---|---|---|---|\n")
        for o in out:
            rd = f"{o['hbm_read_bytes'] / 1e6:.2f}" if o["hbm_read_bytes"] is not None else "-"
            wr = f"{o['hbm_write_bytes'] / 1e6:.2f}" if o["hbm_write_bytes"] is not None else "-"
            f.write(f"| {o['kernel']} | {o['calls']} | {o['avg_us']:.2f} | {o['pct']:.2f} | {rd} | {wr} |\n")
    print(open(os.path.join(dst, "summary.md")).read())


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
