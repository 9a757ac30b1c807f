"""Build libmmni.so (all HIP kernels + the C ABI) in-tree for gfx950.

Invoked by ``__graft_entry__.build()`` and usable directly: ``python -m multimodal_neuroimage_amd.build``.
hipcc cross-compiles for gfx950 without a GPU.  The .so lands next to this file so the
snapshot that travels to the GPU box carries it (git ignores it, gpurun does not).
"""
import os
import subprocess
import sys
import hashlib

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmmni.so")
ARCH = "gfx950"

# -mcode-object-version=5 keeps the code object loadable by the ROCm 7.0 HIP runtime that
# PyTorch bundles (the library resolves libamdhip64.so.7 to torch's copy once torch is loaded).
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}",
         "-mcode-object-version=5", "-Wall", "-Wno-unused-function", "-Wno-unused-result"]


# Per-file extras.  mlp.hip: keep MFMA accumulators in arch VGPRs (the GELU epilogue reads every
# accumulator; AGPR accumulators cost a v_accvgpr_read per element — 323 -> 206 VALU per tile).
# mha.hip: the softmax reads every score accumulator (196 v_accvgpr moves in the bf16 backward).
EXTRA = {f: ["-mllvm", "-amdgpu-mfma-vgpr-form"] for f in ("mlp.hip", "blockops.hip", "mha.hip")}


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _digest():
    h = hashlib.sha256()
    headers = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h"))
    for f in sources() + headers + [os.path.join(HERE, "..", "include", "mmni.h"), __file__]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(FLAGS).encode())
    h.update(repr(sorted(EXTRA.items())).encode())
    return h.hexdigest()


def build(force=False, verbose=True):
    """Compile every csrc/*.hip into libmmni.so; skip when sources are unchanged."""
    stamp = LIB + ".sha256"
    dig = _digest()
    if not force and os.path.exists(LIB) and os.path.exists(stamp):
        with open(stamp) as fh:
            if fh.read().strip() == dig:
                return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs = []
    procs = []
    for src in sources():
        obj = os.path.join("/tmp", "mmni_" + os.path.basename(src) + f".{os.getpid()}.o")
        cmd = [hipcc] + [f for f in FLAGS if f != "-shared"] + EXTRA.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        objs.append(obj)
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{out.decode()}")
        if verbose and out.strip():
            sys.stderr.write(out.decode())
    tmp = LIB + f".tmp{os.getpid()}"
    cmd = [hipcc, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout.decode()}")
    os.replace(tmp, LIB)
    for o in objs:
        try:
            os.remove(o)
        except OSError:
            pass
    with open(stamp, "w") as fh:
        fh.write(dig)
    if verbose:
        sys.stderr.write(f"built {LIB}\n")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
