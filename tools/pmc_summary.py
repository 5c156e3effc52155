#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into profiles/: per-kernel dispatch stats and PMC counters.

Usage:
  tools/pmc_summary.py --workload C4 --command "<cmd>" --out profiles/r04_C4_pmc.json \
      --pmc-dir gpurun_out/pmc_fetch gpurun_out/pmc_write ...
  tools/pmc_summary.py --workload C4 --command "<cmd>" --stats-md profiles/r04_C4_kernel_stats.md \
      --trace-dir gpurun_out/prof

Round-3 builds ran each loop NN search as two grids on two streams (k_nn_group<D>,
k_nn_single<D>); for such traces the stats summary also lists the SPAN of each launch pair,
first start to last end.  Since round 4 the search is one grid (k_nn_search<D>).

Each --pmc-dir holds one separate `rocprofv3 --pmc <counters> --output-format csv` pass
(FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).  HBM bytes per launch:
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, with the raw (1 x FETCH_SIZE) figure
beside it.  The factor 2 is calibrated for every access pattern the kernels use
(tools/fetch_calib.hip, profiles/r05_fetch_calib.json): on gfx950 every fabric read is a
128-B request (TCC_EA0_RDREQ_128B = TCC_EA0_RDREQ; the 32-B / 64-B counts and TCC_BUBBLE
read 0), and FETCH_SIZE = (RDREQ - BUBBLE - RDREQ_32B) x 64 B counts each at 64 B -- so
FETCH_SIZE is exactly half the request bytes for a coalesced 16-B stream and for scattered
4-, 8-, 16- and 48-B gathers alike (TCC_EA0_RDREQ_DRAM_32B x 32 B agrees).  A scattered
gather costs 128 B of fabric traffic per line it touches, whatever its width.
"""
import argparse
import collections
import csv
import glob
import json
import os


def _rows(d, pattern):
    for f in sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True)):
        with open(f, newline="") as fh:
            yield from csv.DictReader(fh)


def pmc(dirs):
    # kernel -> counter -> list of per-dispatch values
    acc = collections.defaultdict(lambda: collections.defaultdict(dict))
    for d in dirs:
        for r in _rows(d, "*counter_collection.csv"):
            k = r.get("Kernel_Name", "?")
            disp = (d, r.get("Dispatch_Id"))
            c = r.get("Counter_Name")
            acc[k][c][disp] = acc[k][c].get(disp, 0.0) + float(r.get("Counter_Value", 0) or 0)
    out = {}
    for k, cs in acc.items():
        means = {c: sum(v.values()) / max(1, len(v)) for c, v in cs.items()}
        nd = max(len(v) for v in cs.values())
        e = {"dispatches": nd, "counters_per_dispatch": means}
        if "FETCH_SIZE" in means and "WRITE_SIZE" in means:
            e["fetch_bytes_raw"] = means["FETCH_SIZE"] * 1024.0
            e["fetch_bytes_corrected"] = 2.0 * means["FETCH_SIZE"] * 1024.0
            e["write_bytes"] = means["WRITE_SIZE"] * 1024.0
            e["hbm_bytes_per_launch_raw"] = e["fetch_bytes_raw"] + e["write_bytes"]
            e["hbm_bytes_per_launch"] = e["fetch_bytes_corrected"] + e["write_bytes"]
        rb = read_bytes_by_size(means)
        if rb:
            # the request-size counters (calibrated on tools/fetch_calib.hip, profiles/r05_fetch_calib.json)
            for name, b in rb.items():
                e[f"fetch_bytes_{name}"] = b
            if "WRITE_SIZE" in means and "dram_32b_units" in rb:
                e["hbm_bytes_per_launch_dram32"] = rb["dram_32b_units"] + means["WRITE_SIZE"] * 1024.0
        if "SQ_WAVE_CYCLES" in means and means["SQ_WAVE_CYCLES"] > 0:
            wc = means["SQ_WAVE_CYCLES"]
            e["frac_wait_any"] = means.get("SQ_WAIT_ANY", 0.0) / wc
            e["frac_wait_inst_any"] = means.get("SQ_WAIT_INST_ANY", 0.0) / wc
            e["frac_active_inst_any"] = means.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
        out[k] = e
    return out


# request-size TCC counters (rocprofv3 counter_defs.yaml, gfx950 events 42-45, 62, 108, 112)
TCC_REQ = ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum",
           "TCC_BUBBLE_sum", "TCC_EA0_RDREQ_DRAM_32B_sum", "TCC_EA0_RDREQ_DRAM_sum"]


def read_bytes_by_size(c):
    """Fabric read bytes from the request-size counters of one dispatch (None if absent):
    32 x 32-B + 64 x 64-B + 128 x 128-B requests, and 32 x the DRAM 32-B units."""
    out = {}
    if all(k in c for k in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")):
        out["by_request_size"] = (32.0 * c["TCC_EA0_RDREQ_32B_sum"] + 64.0 * c["TCC_EA0_RDREQ_64B_sum"]
                                  + 128.0 * c["TCC_EA0_RDREQ_128B_sum"])
    if "TCC_EA0_RDREQ_DRAM_32B_sum" in c:
        out["dram_32b_units"] = 32.0 * c["TCC_EA0_RDREQ_DRAM_32B_sum"]
    return out


def calib(plain_jsonl, dirs):
    """tools/fetch_calib.hip: per access pattern, the counters' bytes against the known
    requested bytes and access count (the timed, second dispatch of each kernel)."""
    known = {}
    for line in open(plain_jsonl):
        line = line.strip()
        if line.startswith("{"):
            d = json.loads(line)
            known[d["kernel"]] = d
    per = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> counter -> dispatch -> value
    for d in dirs:
        for r in _rows(d, "*counter_collection.csv"):
            k = r.get("Kernel_Name", "?").split("(")[0].replace("void ", "").strip()
            per[k][r.get("Counter_Name")][(d, int(r.get("Dispatch_Id", 0)))] = float(r.get("Counter_Value", 0) or 0)
    out = {}
    for k, kn in known.items():
        cs = per.get(k, {})
        c = {}
        for name, disp in cs.items():
            vals = [v for _, v in sorted(disp.items(), key=lambda kv: kv[0][1])]
            c[name] = vals[-1]  # the timed launch (the first one warms page tables)
        req = kn["requested_bytes"]
        e = {"accesses": kn["accesses"], "requested_bytes": req, "ms": kn["ms"], "requested_GBps": kn["requested_GBps"],
             "counters": c}
        if "FETCH_SIZE" in c:
            fb = c["FETCH_SIZE"] * 1024.0
            e["fetch_size_bytes"] = fb
            e["fetch_size_over_requested"] = round(fb / req, 4)
            e["fetch_size_bytes_per_access"] = round(fb / kn["accesses"], 2)
        for name, b in read_bytes_by_size(c).items():
            e[f"bytes_{name}"] = b
            e[f"bytes_{name}_over_requested"] = round(b / req, 4)
            e[f"bytes_{name}_per_access"] = round(b / kn["accesses"], 2)
            e[f"GBps_{name}"] = round(b / (kn["ms"] * 1e-3) / 1e9, 1)
            if "fetch_size_bytes" in e and e["fetch_size_bytes"] > 0:
                e[f"correction_{name}_over_fetch_size"] = round(b / e["fetch_size_bytes"], 4)
        out[k] = e
    return out


def stats_md(dirs):
    agg = collections.defaultdict(list)
    spans = collections.defaultdict(list)  # kernel -> [(start, end)] in time order
    for d in dirs:
        for r in _rows(d, "*kernel_trace.csv"):
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            agg[r["Kernel_Name"]].append(t1 - t0)
            spans[r["Kernel_Name"]].append((t0, t1))
    tot = sum(sum(v) for v in agg.values()) or 1
    lines = ["| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| `{k[:110]}` | {len(v)} | {sum(v) / 1e6:.3f} | {sum(v) / len(v) / 1e3:.2f} | "
                     f"{100.0 * sum(v) / tot:.1f} |")
    out = "\n".join(lines) + "\n"
    pair_lines = []
    for D in (12, 3):
        g = sorted(v for k, vs in spans.items() if f"k_nn_group<{D}>" in k for v in vs)
        s = sorted(v for k, vs in spans.items() if f"k_nn_single<{D}>" in k for v in vs)
        if not g or len(g) != len(s):
            continue
        sp = [max(a[1], b[1]) - min(a[0], b[0]) for a, b in zip(g, s)]
        ov = [max(0, min(a[1], b[1]) - max(a[0], b[0])) for a, b in zip(g, s)]
        pair_lines.append(f"| k_nn_group<{D}> + k_nn_single<{D}> | {len(sp)} | {sum(sp) / 1e6:.3f} | "
                          f"{sum(sp) / len(sp) / 1e3:.2f} | {sum(ov) / len(ov) / 1e3:.2f} |")
    if pair_lines:
        out += ("\n## NN launch pairs (group grid + single-query grid on two streams)\n\n"
                "span = last end - first start of the n-th dispatch of each kernel; overlap = time both ran\n\n"
                "| launch pair | pairs | total span ms | avg span us | avg overlap us |\n|---|---:|---:|---:|---:|\n"
                + "\n".join(pair_lines) + "\n")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pmc-dir", nargs="*", default=[])
    ap.add_argument("--out")
    ap.add_argument("--trace-dir", nargs="*", default=[])
    ap.add_argument("--stats-md")
    ap.add_argument("--command", default="")
    ap.add_argument("--calib", nargs="*", default=None,
                    help="<calib_plain.jsonl> <pmc dirs...>: summarise tools/fetch_calib.sh into --out")
    ap.add_argument("--workload", default="C4", help="bench.py --workload of the profiled command (bench.py keys "
                                                      "the PMC lookups by it)")
    a = ap.parse_args()
    if a.calib:
        res = {"command": a.command or "tools/fetch_calib.sh", "table_bytes": 1 << 30,
               "note": "per pattern: the known accesses / requested bytes of tools/fetch_calib.hip against FETCH_SIZE and "
                       "the TCC request-size counters of the same (second, timed) dispatch",
               "patterns": calib(a.calib[0], a.calib[1:])}
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)
        print(f"wrote {a.out}")
        return
    if a.out:
        res = {"command": a.command, "workload": a.workload, "passes": a.pmc_dir,
               "hbm_formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes (gfx950 FETCH_SIZE reports 1/2)",
               "kernels": pmc(a.pmc_dir)}
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)
        print(f"wrote {a.out}: {len(res['kernels'])} kernels")
    if a.stats_md:
        with open(a.stats_md, "w") as f:
            f.write(f"# rocprofv3 --kernel-trace --stats ({a.workload})\n\ncommand: `{a.command}`\n\n"
                    + stats_md(a.trace_dir))
        print(f"wrote {a.stats_md}")


if __name__ == "__main__":
    main()
