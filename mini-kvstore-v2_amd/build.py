"""Build the native libraries in-tree (they travel to the GPU box with the repo snapshot).

  lib/libkvreplay.so   HIP kernels + the C ABI of include/kvreplay.h   (hipcc, gfx950)
  lib/libkvhost.so     discovery, generator, fold, KVStore mirror      (g++, links libkvreplay)
  ../oracle/liboracle.so   CPU restatement used only by tests / bench cpu_baseline (gcc)
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB = os.path.join(PKG, "lib")
CSRC = os.path.join(PKG, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KVR_OFFLOAD_ARCH", "gfx950")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build failed: " + " ".join(cmd))


def _deps(*names):
    inc = os.path.join(ROOT, "include")
    out = [os.path.join(CSRC, n) for n in names]
    out += [os.path.join(inc, f) for f in os.listdir(inc)]
    return out


def build(force=False, verbose=False):
    os.makedirs(LIB, exist_ok=True)
    rep = os.path.join(LIB, "libkvreplay.so")
    deps = _deps(*[f for f in os.listdir(CSRC) if f.endswith((".hip", ".h"))])
    if force or _newer(rep, deps):
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
              "-Wall", "-Wno-unused-result", "-o", rep, os.path.join(CSRC, "kvr_api.hip")])
        if verbose:
            print("built", rep)
    host = os.path.join(LIB, "libkvhost.so")
    deps = _deps("kvr_host.cpp", "kvr_gen_common.h") + [rep]
    if force or _newer(host, deps):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-o", host,
              os.path.join(CSRC, "kvr_host.cpp"), "-L", LIB, "-lkvreplay",
              "-Wl,-rpath,$ORIGIN", "-Wl,--no-as-needed"])
        if verbose:
            print("built", host)
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    src = os.path.join(ROOT, "oracle", "replay_ref.c")
    if force or _newer(orc, [src, os.path.join(ROOT, "include", "kvreplay.h")]):
        _run(["gcc", "-O3", "-std=c11", "-fPIC", "-shared", "-Wall", "-o", orc, src])
        if verbose:
            print("built", orc)
    return rep, host, orc


def build_prof():
    """Diagnostic variant with per-phase cycle stamps (tools/prof_phases.py); not shipped."""
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, "libkvreplay_prof.so")
    deps = _deps(*[f for f in os.listdir(CSRC) if f.endswith((".hip", ".h"))])
    if _newer(out, deps):
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-DKVR_PROF",
              "-Wno-unused-result", "-o", out, os.path.join(CSRC, "kvr_api.hip")])
    return out


def build_ablate(masks=(0, 1, 2, 3, 7, 8, 16, 32, 64)):
    """Diagnostic variants with parts of k_replay switched off (tools/ablate.py); not shipped."""
    out = os.path.join(LIB, "ablate")
    os.makedirs(out, exist_ok=True)
    deps = _deps(*[f for f in os.listdir(CSRC) if f.endswith((".hip", ".h"))])
    procs = []
    for m in masks:
        so = os.path.join(out, f"libkvreplay_a{m}.so")
        if _newer(so, deps):
            procs.append(subprocess.Popen([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
                                           f"-DKVR_ABLATE={m}", "-Wno-unused-result", "-o", so,
                                           os.path.join(CSRC, "kvr_api.hip")]))
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("ablation build failed")
    return out


# experimental k_replay variants (tools/ablate.py <cfg> 0 <name>): timing only, never shipped.
# Each entry is the -D flags of one build; the kernel's own comments say what each macro does.
VARIANTS = {
    "rt768": ["-DKVR_RT=768"],     # 12 stripes per workgroup
    "prio0": ["-DKVR_HOP_PRIO=0", "-DKVR_REC_PRIO=0"],   # no raised wave priority
    "fin0": ["-DKVR_FIN_PRIO=0"],  # the scan + finalize chain at priority 0
    "lf0": ["-DKVR_LANEFRAME=0"],  # the scalar hop loop for every record
    "a7": ["-DKVR_ABLATE=7"],      # loads + per-tile bookkeeping only (the memory floor at 16 waves/CU)
    "top": ["-DKVR_TOPWAIT=1"],    # wait for the tile's load at the loop top (round 3 default before)
    "bo4": ["-DKVR_FAST_BACKOFF=4"],     # 4 tiles of scalar hops after a short lane-parallel round
    "nouni": ["-DKVR_UNIFOLD=0"],  # long-value views through LDS marks + lane permutes only
    "base": [],
    "u1": ["-DKVR_FP_U=1"],      # k_fold_lds: one record per thread and step
    "u2": ["-DKVR_FP_U=2"],
    "fp4": ["-DKVR_FP_PER=4"],   # k_fold_part: 4 tuples per thread (4096-record regions; neutral)
    # k_piece's workgroup x piece buffers (round 6): 16 waves x 1 buffer is round 5's kernel
    "p1024x1": ["-DKVR_PNT=1024", "-DKVR_PNB=1"],
    "p1024x2": ["-DKVR_PNT=1024", "-DKVR_PNB=2"],
    "p512x2": ["-DKVR_PNT=512", "-DKVR_PNB=2"],
    "p512x3": ["-DKVR_PNT=512", "-DKVR_PNB=3"],
    # k_piece ablations (KVR_PABLATE: results wrong by design, timing only)
    "pa1": ["-DKVR_PABLATE=1"], "pa2": ["-DKVR_PABLATE=2"], "pa11": ["-DKVR_PABLATE=11"],
    "pa16": ["-DKVR_PABLATE=16"], "pa59": ["-DKVR_PABLATE=59"], "pnb": ["-DKVR_PBAL=0"],
    "pa128": ["-DKVR_PABLATE=128"], "pch4": ["-DKVR_PCHAINS=4"], "pwe1": ["-DKVR_PWEARLY=1"], "pa256": ["-DKVR_PABLATE=256"], "pa512": ["-DKVR_PABLATE=512"],
    "pa1536": ["-DKVR_PABLATE=1536"], "pa1920": ["-DKVR_PABLATE=1920"],
    "pa2048": ["-DKVR_PABLATE=2048"], "pa4096": ["-DKVR_PABLATE=4096"], "pw1": ["-DKVR_PWIDE=1", "-DKVR_PRUNFORM=0"], "prf0": ["-DKVR_PRUNFORM=0"], "pdef0": ["-DKVR_PDEFER=0"], "pa32768": ["-DKVR_PABLATE=32768"],
    "pbd32": ["-DKVR_PBAL_D=32"], "pbd128": ["-DKVR_PBAL_D=128"], "pbe2": ["-DKVR_PBAL_EVERY=2"], "pa8192": ["-DKVR_PABLATE=8192"], "pa16384": ["-DKVR_PABLATE=16384"],
    # header windows (round 6): through registers after the CRC (the form before KVR_PWDMA), the DMA
    # windows after the next pieces, the flush waiting vmcnt(0) (profiles/r06/ab_windows_dma.txt)
    "pwdma0": ["-DKVR_PWDMA=0"], "pwaft": ["-DKVR_PWDMA_AFTER=1"], "pwvmc0": ["-DKVR_PWDMA_VMC=0"],
}


def build_variants(names=None):
    out = os.path.join(LIB, "variants")
    os.makedirs(out, exist_ok=True)
    deps = _deps(*[f for f in os.listdir(CSRC) if f.endswith((".hip", ".h"))])
    procs = []
    for n in names or VARIANTS:
        so = os.path.join(out, f"libkvreplay_{n}.so")
        if _newer(so, deps):
            procs.append(subprocess.Popen([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
                                           *VARIANTS[n], "-Wno-unused-result", "-o", so,
                                           os.path.join(CSRC, "kvr_api.hip")]))
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("variant build failed")
    return out


def build_variant_pair(name):
    """lib/vpair/<name>/: a VARIANTS build of libkvreplay.so with its own libkvhost.so, so a whole
    process (kvreplay with KVREPLAY_VARIANT=<name>) runs the variant; timing tools only."""
    out = os.path.join(LIB, "vpair", name)
    os.makedirs(out, exist_ok=True)
    rep = os.path.join(out, "libkvreplay.so")
    deps = _deps(*[f for f in os.listdir(CSRC) if f.endswith((".hip", ".h"))])
    if _newer(rep, deps):
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", *VARIANTS[name],
              "-Wno-unused-result", "-o", rep, os.path.join(CSRC, "kvr_api.hip")])
    host = os.path.join(out, "libkvhost.so")
    if _newer(host, _deps("kvr_host.cpp", "kvr_gen_common.h") + [rep]):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", host, os.path.join(CSRC, "kvr_host.cpp"),
              "-L", out, "-lkvreplay", "-Wl,-rpath,$ORIGIN", "-Wl,--no-as-needed"])
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    if "--prof" in sys.argv:
        print("built", build_prof())
    if "--ablate" in sys.argv:
        print("built", build_ablate())
    if "--variants" in sys.argv:
        print("built", build_variants())
