"""Build libaiyagari.so (hand-written HIP for gfx950) in-tree.

``python -m aiyagari_hark_amd.build`` compiles ``csrc/*.hip`` with hipcc (one object per
translation unit, in parallel) and links ``aiyagari_hark_amd/lib/libaiyagari.so``.  The
shared object is git-ignored but travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libaiyagari.so")
SOURCES = ["api.hip", "index.hip", "egm.hip", "panel_tab.hip", "panel.hip", "panel_block.hip", "panel_resident.hip",
           "hist.hip", "hist_resident.hip", "hist_krylov.hip", "stats.hip", "ge.hip", "ge_resident.hip", "hooks.hip"]
HEADERS = ["common.h", "internal.h", "panel_common.h", "hist_cluster.h", "egm_common.h", "hist_bicg.h", "ge_search.h",
           "hist_pull.h"]
ARCH = os.environ.get("AIY_OFFLOAD_ARCH", "gfx950")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-munsafe-fp-atomics", "-Wall", "-Wno-unused-result",
          "-I/opt/rocm/include"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found; the MI355X build needs ROCm's hipcc")


def sources():
    return [f for f in SOURCES if os.path.exists(os.path.join(CSRC, f))]


def source_digest() -> str:
    """sha256 (first 16 hex digits) of every source the library is built from (csrc/*, the
    ABI header): profiles/pmc_traffic.json stamps each PMC pass with it, and bench.py
    reports a pass's traffic only while the sources are still the ones profiled."""
    import hashlib
    hsh = hashlib.sha256()
    files = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".h")))
    for f in files:
        hsh.update(f.encode())
        hsh.update(open(os.path.join(CSRC, f), "rb").read())
    hsh.update(open(os.path.join(HERE, "..", "include", "aiyagari.h"), "rb").read())
    return hsh.hexdigest()[:16]


def needs_rebuild() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in sources() + HEADERS]
    deps.append(os.path.join(HERE, "..", "include", "aiyagari.h"))
    return (any(os.path.getmtime(d) > t for d in deps if os.path.exists(d)) or
            library_digest(LIB) != source_digest())


def build(force: bool = False, verbose: bool = True, out: str = LIB, defines=()) -> str:
    if out == LIB and not force and not needs_rebuild():
        return LIB
    os.makedirs(os.path.dirname(out), exist_ok=True)
    objdir = out + ".objs"
    os.makedirs(objdir, exist_ok=True)
    cc = hipcc()
    flags = [f"--offload-arch={ARCH}"] + CFLAGS + [f"-D{d}" for d in defines]

    # objects are kept next to the library and rebuilt only when their source, a header or the
    # flags changed (a header change rebuilds everything)
    stamp = os.path.join(objdir, "flags.txt")
    same_flags = os.path.exists(stamp) and open(stamp).read() == " ".join(flags)
    hdr_t = max([os.path.getmtime(os.path.join(CSRC, f)) for f in HEADERS if os.path.exists(os.path.join(CSRC, f))] +
                [os.path.getmtime(os.path.join(HERE, "..", "include", "aiyagari.h"))])

    def compile_one(src):
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        if (same_flags and not force and os.path.exists(obj) and
                os.path.getmtime(obj) > max(hdr_t, os.path.getmtime(os.path.join(CSRC, src)))):
            return obj
        cmd = [cc] + flags + ["-c", os.path.join(CSRC, src), "-o", obj + ".tmp.o"]
        if verbose:
            print("[aiyagari build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp.o", obj)
        return obj

    if not same_flags:
        open(stamp, "w").write(" ".join(flags))
    jobs = min(len(sources()), max(1, min(16, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, sources()))
    tmp = out + ".tmp"
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC"] + objs + ["-L/opt/rocm/lib", "-lrccl", "-o", tmp]
    if verbose:
        print("[aiyagari build]", " ".join(cmd), flush=True)
    # computed before linking: the sources this library was built from (+ any diagnostic defines,
    # so a variant build never passes for the product library)
    digest = source_digest() + ("+" + ",".join(defines) if defines else "")
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    # sidecar: the source digest the library was built from (tools/prof_bench.sh stamps a PMC
    # pass with the digest of the library the bench actually loads, not just of the sources)
    with open(out + ".digest", "w") as f:
        f.write(digest + "\n")
    return out


def library_digest(path: str = LIB):
    """The source digest a built library was made from (its .digest sidecar), or None."""
    try:
        return open(path + ".digest").read().strip() or None
    except OSError:
        return None


def build_variant(name: str, defines) -> str:
    """Diagnostic / tuning build (tools/panel_variants.py): lib/variants/libaiyagari_<name>.so
    with extra preprocessor defines; never loaded by the product path."""
    return build(out=os.path.join(LIBDIR, "variants", f"libaiyagari_{name}.so"), defines=defines)


if __name__ == "__main__":
    # python -m aiyagari_hark_amd.build [--force] | --variant NAME DEFINE [DEFINE ...]
    if "--variant" in sys.argv:
        i = sys.argv.index("--variant")
        print(build_variant(sys.argv[i + 1], sys.argv[i + 2:]))
    else:
        build(force="--force" in sys.argv)
        print(LIB)
