"""HBM traffic of k_replay's main pass from PMC counters (run on the GPU box).

Two rocprofv3 passes over a short bench run (FETCH_SIZE and WRITE_SIZE cannot share a pass on
gfx950), corrected as MI355X_MICROARCH.md §HBM prescribes: WRITE_SIZE is in KiB (x 1024);
FETCH_SIZE is in KiB and its byte factor depends on the access width (x 2 only for 16-B/lane
coalesced streams), so a third pass calibrates it on k_replay's own load pattern: the loads-only
build (KVR_ABLATE=64) over a known byte count.
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


def run_pass(counter, args, tag=None, prog=None):
    d = os.path.join(OUT, tag or counter)
    os.makedirs(d, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
           sys.executable, prog or os.path.join(ROOT, "bench.py")] + args
    with open(os.path.join(d, "log.txt"), "w") as log:
        subprocess.run(cmd, check=True, cwd="/tmp", env=env, stdout=log, stderr=subprocess.STDOUT, timeout=600)
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if "k_replay" in r["Kernel_Name"]]
    main = max(int(r["Grid_Size"]) for r in rows)          # the first pass (re-walk passes are smaller)
    vals = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) == main]
    return sum(vals) / len(vals), len(vals)


def calibrate():
    """FETCH_SIZE bytes-per-KiB of k_replay's own load pattern (MI355X_MICROARCH.md: widths other
    than 16 B/lane coalesced are uncalibrated): the loads-only build (KVR_ABLATE=64) reads every
    segment byte of cfg2 exactly once, so known bytes / (KiB x 1024) is the factor."""
    kib, _ = run_pass("FETCH_SIZE", ["cfg2", "0", "64"], tag="calib", prog=os.path.join(ROOT, "tools", "ablate.py"))
    log = open(os.path.join(OUT, "calib", "log.txt")).read()
    known = int(log.split("seg_bytes=")[1].split()[0])
    return known / (kib * 1024), kib, known


def main():
    args = sys.argv[1:] or ["--steps", "2", "--warmup", "1", "--no-cpu", "--no-stream", "--no-open"]
    factor, calib_kib, calib_bytes = calibrate()
    fetch_kib, nf = run_pass("FETCH_SIZE", args)
    write_kib, nw = run_pass("WRITE_SIZE", args)
    res = {"kernel": "k_replay", "lib_sha256_16": lib_hash(), "bench_args": args,
           "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib,
           "fetch_calibration": {"kernel": "k_replay KVR_ABLATE=64 (loads only)", "known_bytes": calib_bytes,
                                 "fetch_size_kib_raw": calib_kib, "bytes_per_kib": factor * 1024},
           "hbm_read_bytes": fetch_kib * 1024 * factor, "hbm_write_bytes": write_kib * 1024,
           "dispatches": [nf, nw],
           "correction": "FETCH_SIZE KiB x1024 x (calibrated factor of this load pattern, measured on the "
                         "loads-only build over a known byte count), WRITE_SIZE KiB x1024"}
    res["hbm_bytes"] = res["hbm_read_bytes"] + res["hbm_write_bytes"]
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    res["run_dir"] = os.path.relpath(OUT, ROOT)
    with open(os.path.join(ROOT, "gpurun_out", "pmc_traffic.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
