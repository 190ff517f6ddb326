"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR BENCH_JSON OUT_JSON

Both passes run `bench.py ... --pmc-target R`: after its timing, bench
re-issues the dominant kernel's main launch R times, so the LAST R
dispatches of that kernel name in each counter CSV are exactly that launch
shape; their mean FETCH_SIZE / WRITE_SIZE is its HBM traffic per launch.
FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the
bytes of wide (16 B/lane) coalesced reads (MI355X_MICROARCH.md, HBM section),
so reads are doubled; WRITE_SIZE is exact for the kernels' 4-16 B/lane stores.
The table is merged into OUT_JSON under "<kernel>|<shape>" (bench.py's
traffic_lookup key), plus a per-kernel-name mean over every dispatch.
"""
import collections
import csv
import json
import os
import re
import sys


def rows(path, counter):
    out = []
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            out.append((int(r.get("Dispatch_Id", 0) or 0), short(r["Kernel_Name"]), float(r["Counter_Value"])))
    out.sort()
    return out


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(sgg::[A-Za-z_0-9:]+(<[^()]*>)?)\(", name)
    return m.group(1) if m else name[:60]


def main():
    fdir, wdir, bench, out = sys.argv[1:5]
    fr, wr = rows(fdir, "FETCH_SIZE"), rows(wdir, "WRITE_SIZE")
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    tgt = line["pmc_target"]
    name, reps = tgt["kernel"], tgt["reps"]
    res = json.load(open(out)) if os.path.exists(out) else {}
    res["source"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate runs) of `bench.py --pmc-target R`; "
                     "the last R dispatches of the target kernel; FETCH_SIZE x2 (gfx950)")
    base = name.split("+")[0]
    match = (lambda k: k == base) if "<" in base else (lambda k: k.split("<")[0] == base)
    f_t = [v for _, k, v in fr if match(k)][-reps:]
    w_t = [v for _, k, v in wr if match(k)][-reps:]
    wt = json.loads(open(bench.replace("fetch", "write")).read().strip().splitlines()[-1]).get("pmc_target") \
        if "fetch" in bench and os.path.exists(bench.replace("fetch", "write")) else tgt
    if wt != tgt:
        raise SystemExit("the FETCH and WRITE passes re-issued different launches: %s vs %s" % (tgt, wt))
    rd = 2.0 * 1024.0 * sum(f_t) / max(len(f_t), 1)
    wb = 1024.0 * sum(w_t) / max(len(w_t), 1)
    res["%s|%s" % (name, tgt["shape"])] = {"read_bytes": rd, "write_bytes": wb, "hbm_bytes": rd + wb,
                                           "dispatches": len(f_t)}
    per = collections.defaultdict(list)
    for _, k, v in fr:
        per[k].append(v)
    perw = collections.defaultdict(list)
    for _, k, v in wr:
        perw[k].append(v)
    res["kernels"] = {k: {"read_bytes": 2048.0 * sum(v) / len(v),
                          "write_bytes": 1024.0 * sum(perw.get(k, [0.0])) / max(len(perw.get(k, [])), 1),
                          "dispatches": len(v)} for k, v in per.items()}
    for k in res["kernels"]:
        res["kernels"][k]["hbm_bytes"] = res["kernels"][k]["read_bytes"] + res["kernels"][k]["write_bytes"]
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res["%s|%s" % (name, tgt["shape"])], indent=1))


if __name__ == "__main__":
    main()
