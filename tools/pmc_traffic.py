"""HBM traffic of one replay (k_piece + k_replay's main pass) from PMC counters (run on the GPU box).

Two rocprofv3 passes over a short bench run (FETCH_SIZE and WRITE_SIZE cannot share a pass on
gfx950), corrected as MI355X_MICROARCH.md §HBM prescribes: WRITE_SIZE is in KiB (x 1024);
FETCH_SIZE is in KiB and its byte factor depends on the access width (x 2 only for 16-B/lane
coalesced streams), so a third pass calibrates it on k_piece's own load pattern: tools/piece_probe
calib (dword-aligned 16-B loads of 128-B pieces, lane l at piece l, cfg2's record geometry) over a
known byte count.
Writes profiles/pmc_traffic.json, keyed by the hash of the libkvreplay.so it measured, which
bench.py reports as roofline.traffic when the library still matches.

  python tools/pmc_traffic.py [bench args...]
"""
import csv
import glob
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mini-kvstore-v2_amd", "lib", "libkvreplay.so")
# every run keeps its own rocprofv3 output and logs (a failed pass's cause survives later runs)
OUT = os.path.join(ROOT, "gpurun_out", "pmc_traffic", time.strftime("%Y%m%d-%H%M%S"))


def lib_hash():
    return hashlib.sha256(open(LIB, "rb").read()).hexdigest()[:16]


def run_pass(counter, args, tag=None, prog=None, kernels=("k_piece", "k_replay")):
    """-> ({kernel: mean counter value of its main dispatch}, stdout of the program)"""
    d = os.path.join(OUT, tag or counter)
    os.makedirs(d, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    target = [prog] if prog and not prog.endswith(".py") else [sys.executable, prog or os.path.join(ROOT, "bench.py")]
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--"] + target + args
    with open(os.path.join(d, "log.txt"), "w") as log:
        subprocess.run(cmd, check=True, cwd="/tmp", env=env, stdout=log, stderr=subprocess.STDOUT, timeout=600)
    res = {}
    for kern in kernels:
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            rows += [r for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"]]
        if not rows:
            continue
        main = max(int(r["Grid_Size"]) for r in rows)          # the first pass (re-walk passes are smaller)
        vals = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) == main]
        res[kern] = (sum(vals) / len(vals), len(vals))
    return res, open(os.path.join(d, "log.txt")).read()


def calibrate():
    """FETCH_SIZE bytes-per-KiB of k_piece's load pattern (MI355X_MICROARCH.md: widths other than
    16 B/lane coalesced are uncalibrated): tools/piece_probe calib reads a known byte count with the
    same dword-aligned piece loads."""
    r, log = run_pass("FETCH_SIZE", ["calib"], tag="calib", prog=os.path.join(ROOT, "tools", "piece_probe"),
                      kernels=("k_pat",))
    kib = r["k_pat"][0]
    known = int(log.split("calib_bytes_per_dispatch=")[1].split()[0])
    return known / (kib * 1024), kib, known


def main():
    args = sys.argv[1:] or ["--steps", "2", "--warmup", "1", "--no-cpu", "--no-stream", "--no-open"]
    factor, calib_kib, calib_bytes = calibrate()
    fr, _ = run_pass("FETCH_SIZE", args)
    wr, _ = run_pass("WRITE_SIZE", args)
    fetch_kib = sum(v for v, _ in fr.values())
    write_kib = sum(v for v, _ in wr.values())
    res = {"kernel": " + ".join(fr), "lib_sha256_16": lib_hash(), "bench_args": args,
           "fetch_size_kib_raw": {k: v for k, (v, _) in fr.items()},
           "write_size_kib_raw": {k: v for k, (v, _) in wr.items()},
           "fetch_calibration": {"kernel": "tools/piece_probe calib (k_pat<2,2>: k_piece's piece loads)",
                                 "known_bytes": calib_bytes, "fetch_size_kib_raw": calib_kib,
                                 "bytes_per_kib": factor * 1024},
           "hbm_read_bytes": fetch_kib * 1024 * factor, "hbm_write_bytes": write_kib * 1024,
           "dispatches": {k: n for k, (_, n) in fr.items()},
           "correction": "FETCH_SIZE KiB x1024 x (calibrated factor of the piece load pattern, measured by "
                         "tools/piece_probe over a known byte count), WRITE_SIZE KiB x1024; per replay = "
                         "k_piece's dispatch + k_replay's main dispatch"}
    res["hbm_bytes"] = res["hbm_read_bytes"] + res["hbm_write_bytes"]
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    res["run_dir"] = os.path.relpath(OUT, ROOT)
    with open(os.path.join(ROOT, "gpurun_out", "pmc_traffic.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
