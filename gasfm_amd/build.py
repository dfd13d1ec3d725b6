"""In-tree build of libgasfm.so (HIP, gfx950) — no JIT cache, no site-packages.

``python -m gasfm_amd.build`` or ``__graft_entry__.build()`` compiles every
``gasfm_amd/csrc/*.hip`` / ``*.cpp`` into ``gasfm_amd/libgasfm.so`` with
``hipcc --offload-arch=gfx950``.  The .so is git-ignored but travels to the
GPU box with the repo snapshot.
"""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libgasfm.so")
ARCH = os.environ.get("GASFM_OFFLOAD_ARCH", "gfx950")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def file_flags(src):
    """Extra hipcc flags a source asks for on its first line (``// hipcc-flags: ...``), e.g. the
    machine scheduler of csrc/edge_seam.hip."""
    with open(src) as f:
        first = f.readline()
    tag = "// hipcc-flags:"
    return first[len(tag):].split() if first.startswith(tag) else []


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.hpp")) + [
        os.path.join(HERE, "..", "include", "gasfm.h")]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build(force=False, verbose=False, defines=(), out=None):
    """Compile and link libgasfm.so.  ``defines``/``out`` build an A/B variant (e.g.
    ``defines=["GASFM_FWD_LOOKAHEAD=1"], out=".../libgasfm_la.so"``) that ``GASFM_LIB``
    selects at load time; the default library is untouched."""
    lib = out or LIB
    if out is None and not force and not _stale():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs = []
    tag = "" if out is None else "_" + os.path.splitext(os.path.basename(out))[0]
    build_dir = os.path.join(HERE, "_build" + tag)
    os.makedirs(build_dir, exist_ok=True)
    procs = []
    for src in sources():
        obj = os.path.join(build_dir, os.path.basename(src) + ".o")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-c", src, "-o", obj] + file_flags(src)
        cmd += [f"-D{d}" for d in defines]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        objs.append(obj)
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{out.decode(errors='replace')}")
    tmp = lib + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stdout.decode(errors="replace"))
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
