"""Where the one-kernel tail forward / backward spend their time, phase by phase (diagnostic build).

  python tools/tail_stamps.py build        # here (CPU): hic-gnn_amd/hicgat/libhicgat_stamps.so
  python tools/tail_stamps.py run [world]  # GPU box: rank 0 of the simulated world-rank xagg step
  python tools/tail_stamps.py rows M ...   # GPU box: the plain fused tail (no head GEMMs) on M random rows

``build`` copies csrc/ to /tmp, inserts a stamp (``s_memtime`` by wave 0 of every workgroup, stored
with a per-lane vector store into a debug buffer nothing else reads) at the entry of
tail_fwd_kernel / tail_bwd_kernel, after every ``__syncthreads()`` of their bodies and at their end,
adds ``hicgat_debug_set_stamps(ptr)``, and links the variant library.  ``run`` loads it
(HICGAT_LIB), runs eager steps of rank 0's share and prints, per phase, the median over workgroups
of the cycles between consecutive stamps.  Read the SHARES, not the length: the stamps' waits
forbid overlaps the real kernel has (cdna_hip_programming.md, In-kernel stamps).
"""
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hic-gnn_amd")
LIB = os.path.join(PKG, "hicgat", "libhicgat_stamps.so")
MAXS = 24   # stamps per workgroup

# the debug pointer is read once at the kernel's entry (gs_, a register): re-reading it at each stamp
# would wait vmcnt(0) there and drain the weight ring's loads
STAMP = ('if (gs_ && threadIdx.x < 64) { unsigned long long t_; '
         'asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t_) :: "memory"); '
         'gs_[((size_t)blockIdx.x * ' + str(MAXS) + ' + {k}) * 64 + threadIdx.x] = t_; }')
BASE = {"tail_fwd_kernel": 0, "tail_bwd_kernel": MAXS // 2}


def _kernel_body(src, name):
    i = src.index(f"void {name}(")
    j = src.index(") {", i) + 2
    depth, k = 0, j
    while True:
        c = src[k]
        depth += c == "{"
        depth -= c == "}"
        k += 1
        if depth == 0:
            return j + 1, k - 1


def stamped(src):
    """Stamps at entry, after every __syncthreads() and at the end of the two tail kernels' bodies;
    the forward's in slots [0, MAXS/2), the backward's in [MAXS/2, MAXS)."""
    out, count = src, {}
    for name in ("tail_bwd_kernel", "tail_fwd_kernel"):      # the later one first: offsets stay valid
        b, e = _kernel_body(out, name)
        base, n = BASE[name], [1]

        def rep(m):
            st = m.group(0) + " " + STAMP.replace("{k}", str(base + n[0]))
            n[0] += 1
            return st
        body = re.sub(r"__syncthreads\(\);", rep, out[b:e])
        body = "\n  unsigned long long *const gs_ = g_stamps;\n  " + STAMP.replace("{k}", str(base)) + body + "\n  " + STAMP.replace("{k}", str(base + n[0])) + "\n"
        assert n[0] + 1 <= MAXS // 2, name
        count[name] = n[0] + 1
        out = out[:b] + body + out[e:]
    out = out.replace("namespace hicgat {", "namespace hicgat {\n__device__ unsigned long long *g_stamps = nullptr;", 1)
    out += ('\nextern "C" int hicgat_debug_set_stamps(void *p) {\n'
            '  return hipMemcpyToSymbol(HIP_SYMBOL(hicgat::g_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -2;\n}\n')
    return out, count


def build():
    top = "/tmp/hicgat_stamps"
    shutil.rmtree(top, ignore_errors=True)
    tmp = os.path.join(top, "pkg")       # csrc/common.hpp includes ../../include/hicgat.h
    shutil.copytree(os.path.join(PKG, "csrc"), os.path.join(tmp, "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(top, "include"))
    p = os.path.join(tmp, "csrc", "tail_fused.hip")
    src, count = stamped(open(p).read())
    open(p, "w").write(src)
    objs = []
    for f in sorted(os.listdir(os.path.join(tmp, "csrc"))):
        if not f.endswith(".hip"):
            continue
        o = os.path.join(tmp, f[:-4] + ".o")
        extra = ["-fno-slp-vectorize"] if f == "pairdist.hip" else []
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall",
                        "-Wno-unused-result", *extra, f"-I{os.path.join(ROOT, 'include')}", "-c",
                        os.path.join(tmp, "csrc", f), "-o", o], check=True)
        objs.append(o)
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", *objs, "-o", LIB], check=True)
    print("built", LIB, count)


def run(world):
    os.environ["HICGAT_LIB"] = LIB
    sys.path[:0] = [ROOT, PKG]
    import ctypes

    import numpy as np
    import torch

    import bench
    import hicgat
    from hicgat import _lib
    from hicgat import dist as hdist
    lib = _lib.load()
    fn = lib.hicgat_debug_set_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    wl = bench.build_workload("synth-20000", 0, dev)
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().to(dev)
    tr = hdist.ShardedTrainer(model, wl["x"], wl["adj"], wl["truth"], lr=1e-3, mode="xagg",
                              comm=hdist.SimComm(world, 0))
    tr.opt.enable_device_step()
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    nwg = (tr.local_rows + 15) // 16
    buf = torch.zeros(nwg * MAXS * 64, dtype=torch.int64, device=dev)
    assert fn(ctypes.c_void_p(buf.data_ptr())) == 0
    stamps = []
    for _ in range(5):
        buf.zero_()
        tr.step()
        torch.cuda.synchronize()
        stamps.append(buf.view(nwg, MAXS, 64)[:, :, 0].cpu().numpy().astype(np.float64))
    assert fn(None) == 0
    st = np.stack(stamps)                      # [steps, nwg, MAXS]
    print(f"rank 0 of {world}: {tr.local_rows} rows, {nwg} workgroups of 16 (cycles: s_memtime shader clock)")
    for name, base in BASE.items():
        blk = st[:, :, base:base + MAXS // 2]
        n = int((blk[0, 0] > 0).sum())
        d = np.diff(blk[:, :, :n], axis=2)           # per step, workgroup, phase
        med = np.median(d.reshape(-1, n - 1), axis=0)
        span = np.median(blk[:, :, n - 1] - blk[:, :, 0])
        print(f"{name}: {n} stamps, median workgroup span {span:.0f} cycles")
        for k, v in enumerate(med):
            print(f"  phase {k:2d}: {v:9.0f} cycles  {v / med.sum():6.1%}")


def rows(ms):
    """The fused tail without the head GEMMs on M random rows, forward + backward, for each M: the
    per-phase cycles at M / 16 workgroups -- few workgroups (no chip-wide contention for L2 / fabric)
    against the 169 of a P = 8 rank tell a per-CU bound from a shared one."""
    os.environ["HICGAT_LIB"] = LIB
    os.environ["HICGAT_FUSED_TAIL_MIN_M"] = "1"
    sys.path[:0] = [ROOT, PKG]
    import ctypes

    import numpy as np
    import torch

    import hicgat
    from hicgat import _lib, ops
    lib = _lib.load()
    fn = lib.hicgat_debug_set_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().to(dev)
    for M in ms:
        x = torch.relu(torch.randn(M, 512, device=dev)).requires_grad_(True)
        dc = torch.randn(M, 3, device=dev)
        assert ops.fused_tail_ok(model, x), M

        def step():
            model.zero_grad(set_to_none=False)
            ops.fused_tail(model, x).backward(dc)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        nwg = (M + 15) // 16
        buf = torch.zeros(nwg * MAXS * 64, dtype=torch.int64, device=dev)
        assert fn(ctypes.c_void_p(buf.data_ptr())) == 0
        stamps = []
        for _ in range(5):
            buf.zero_()
            step()
            torch.cuda.synchronize()
            stamps.append(buf.view(nwg, MAXS, 64)[:, :, 0].cpu().numpy().astype(np.float64))
        assert fn(None) == 0
        st = np.stack(stamps)
        print(f"M = {M}: {nwg} workgroups of 16 rows")
        for name, base in BASE.items():
            blk = st[:, :, base:base + MAXS // 2]
            n = int((blk[0, 0] > 0).sum())
            d = np.diff(blk[:, :, :n], axis=2)
            med = np.median(d.reshape(-1, n - 1), axis=0)
            span = np.median(blk[:, :, n - 1] - blk[:, :, 0])
            print(f"  {name}: median span {span:.0f} cycles; phases " + " ".join(f"{v:.0f}" for v in med))


if __name__ == "__main__":
    if sys.argv[1] == "rows":
        rows([int(a) for a in sys.argv[2:]])
        sys.exit(0)
    if sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 8)
