"""The executed-work model of one training iteration from a bench.py JSON
line: per kernel its launches, algorithmic FLOP and bytes per iteration (the
work models bench.py's timer divides by, recovered as rate x time), the
roofline time max(FLOP / 157.3 TFLOP/s, bytes / 8 TB/s) and the measured
time; then the totals per scene against SURVEY.md 8(d)'s reference work.
usage: python tools/iteration_model.py BENCH_JSON [--leg NAME]"""
import json
import sys

PEAK_F, PEAK_B = 157.3e12, 8.0e12
REF_FLOP_PER_SCENE = 2.29e9


def main():
    path = sys.argv[1]
    leg = sys.argv[sys.argv.index("--leg") + 1] if "--leg" in sys.argv else None
    d = json.loads(open(path).read().strip().splitlines()[-1])
    if leg:
        d = {l["config"]: l for l in d["legs"]}[leg]
        scenes = d["scenes_per_gpu"]
    else:
        scenes = d["config"]["global_batch"] // d["n_gpus"]
    rows = []
    if "launch_table" in d and "flop" in d["launch_table"][0]:   # every launch shape, its own work model
        for r in d["launch_table"]:
            n = r["per_iter"]
            roof = n * max(r["flop"] / PEAK_F, r["bytes"] / PEAK_B) * 1e6
            rows.append(("%s %s" % (r["kernel"], r["shape"]), n, n * r["flop"], n * r["bytes"], roof,
                         r["us_per_iter"]))
    else:   # (older lines: the top kernels only, work recovered as rate x time)
        for name, k in d["kernels"].items():
            us = k["us_per_iter"]
            fl = k["TFLOP/s"] * 1e12 * us * 1e-6
            nb = k["GB/s"] * 1e9 * us * 1e-6
            roof = max(fl / PEAK_F, nb / PEAK_B) * 1e6
            rows.append((name, k["launches_per_iter"], fl, nb, roof, us))
    rows.sort(key=lambda r: -r[5])
    print("%-84s %5s %9s %8s %8s %8s" % ("kernel [launch shape]", "n/it", "MFLOP", "MB", "roof_us", "meas_us"))
    for name, n, fl, nb, roof, us in rows:
        print("%-84s %5.1f %9.1f %8.2f %8.2f %8.1f" % (name[:84], n, fl / 1e6, nb / 1e6, roof, us))
    F = sum(r[2] for r in rows)
    Bt = sum(r[3] for r in rows)
    R = sum(r[4] for r in rows)
    M = sum(r[5] for r in rows)
    ms = d["ms_per_step"] * 1e3
    print("total: %.3f GFLOP, %.1f MB, roofline %.1f us, instrumented device %.1f us, measured %.1f us per iteration"
          % (F / 1e9, Bt / 1e6, R, M, ms))
    print("per scene (%d scenes): %.1f MFLOP executed vs %.0f MFLOP reference (SURVEY 8d): x%.1f less work"
          % (scenes, F / scenes / 1e6, REF_FLOP_PER_SCENE / 1e6, REF_FLOP_PER_SCENE * scenes / F))
    print("iteration fraction of roofline: %.3f (roofline time / measured time)" % (R / ms))


if __name__ == "__main__":
    main()
