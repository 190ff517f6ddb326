"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR BENCH_JSON OUT_JSON

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the
bytes of wide (16 B/lane) coalesced reads (MI355X_MICROARCH.md, HBM section),
so reads are doubled; WRITE_SIZE is exact for the kernels' 4-16 B/lane stores.
Output keys are "<kernel>|[bn, gpw, unroll, scenes, peds]" for the pool forward
launches that bench.py reports (matched by kernel name, only where one launch
shape has that name), plus a per-kernel-name table of every kernel.
"""
import collections
import csv
import json
import re
import sys


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path + "/run_counter_collection.csv")):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(sgg::[A-Za-z_0-9:]+(<[^()]*>)?)\(", name)
    return m.group(1) if m else name[:60]


def main():
    fdir, wdir, bench, out = sys.argv[1:5]
    fetch, nf = per_kernel(fdir, "FETCH_SIZE")
    write, _ = per_kernel(wdir, "WRITE_SIZE")
    kernels = {}
    for k in fetch:
        rd = 2.0 * fetch[k] * 1024.0
        wr = write.get(k, 0.0) * 1024.0
        kernels[short(k)] = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr, "dispatches": nf[k]}
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    note = line["roofline"]["note"]
    keys = [json.loads(s) for s in re.findall(r"'(\[[0-9, ]+\])'", note)]
    res = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate runs) of "
                     "`bench.py --steps 2 --warmup 1 --graph 0 --no-cpu-baseline`; FETCH_SIZE x2 (gfx950)",
           "kernels": kernels}
    by_name = collections.defaultdict(list)
    for key in keys:
        by_name["sgg::pool_fwd_kernel<%d, %d, %d>" % tuple(key[:3])].append(key)
    for name, ks in by_name.items():
        if len(ks) == 1 and name in kernels:
            res["%s|%s" % (name, ks[0])] = kernels[name]
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in res.items() if "|" in k}, indent=1))


if __name__ == "__main__":
    main()
