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


# experimental k_replay variants (tools/ablate.py <cfg> 0 <name>): timing only, not shipped
VARIANTS = {
    "rt768": ["-DKVR_RT=768"],
    "rt512": ["-DKVR_RT=512"],
    "v9": ["-DKVR_KERNEL_V9"],
    "v9a3": ["-DKVR_KERNEL_V9", "-DKVR_ABLATE=3"],
    "v9a64": ["-DKVR_KERNEL_V9", "-DKVR_ABLATE=64"],
    "v8": ["-DKVR_KERNEL_V8"],
    "prio0": ["-DKVR_HOP_PRIO=0", "-DKVR_REC_PRIO=0"],   # wave priority off
    "bulklow": ["-DKVR_BULK_LOWPRIO=1"],
    "fin0": ["-DKVR_FIN_PRIO=0"],
    "fin2": ["-DKVR_FIN_PRIO=2"],
    "fin1rp2": ["-DKVR_REC_PRIO=2"],
    "s2": ["-DKVR_S4=0"],
    "kscan": ["-DKVR_XSCAN=0"],
    "hopold": ["-DKVR_HOPFAST=0"],
    "unitsel": ["-DKVR_UNITLITE=0"],
    "nodefer": ["-DKVR_DEFER=0"],
    "foldnokey": ["-DKVR_FOLD_NOKEY"],
    "foldsplit": ["-DKVR_FOLD_MERGE=0"],   # every tag match verified by k_fold_verify   # fold kernels without key reads (timing bound only)   # long-value unit views updated in the hop loop   # unit loop with per-step register/data selects   # the hop loop with its separate range checks   # segmented scan with a multiply at every step   # slice-by-2 unit loop (two LDS round trips per word)
    "pf": ["-DKVR_PF=1"],        # touch load of the next tile before the CRC phase (1.66 vs 1.64 ms, not kept)
    "finr": ["-DKVR_FINR=1"],    # value-end tail bytes in one lookup round (A/B: 1.604 vs 1.589 ms, not kept)
    "hop1": ["-DKVR_HOP2=0"],    # the single exact hop loop for every record (1.642 vs 1.604 ms)
    "late": ["-DKVR_EARLY=0"],   # next tile loaded after the finalize
    "rec1": ["-DKVR_LATEREC=1"],   # the last record batch after the unit loop (A/B 1.689 vs 1.601 ms: not kept)
    "tres0": ["-DKVR_TRES_EARLY=0"],   # TileRes stored at the end of the tile
    "cmp32": ["-DKVR_COMPACT16=0", "-DKVR_CSTRIPE=0"],   # k_compact with one 32-B tuple per thread
    "ctile": ["-DKVR_CSTRIPE=0"],   # compaction by 256-tile blocks after a scan of tile counts
    "xf1": ["-DKVR_XFUSE=1"],   # unit-loop registers as two XOR terms (A/B 1.661 vs 1.579 ms: not kept)
    "base": [],
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
