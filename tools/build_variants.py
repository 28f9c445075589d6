"""Build-time variants of the single-deployment kernel (D1_*_V macros in
rollout_d1.hip: D1_S_V quiet steps per iteration, D1_K_V event cadence,
D1_VMN_V trace rows in flight, D1_LEAN_V default-behavior quiet path, D1_NT_V /
D1_NTL_V streaming hints) as separate libccka.so copies under csrc/build/variants/<name>/,
linked with the main build's other objects. Profiling aid only.
NAME=r@other.hip replaces rollout.hip (the general kernel) instead, NAME=p@other.hip pg.hip, NAME=m@other.hip
mlp.hip (NAME=m@mlp.hip:-DX builds mlp.hip itself with extra flags), NAME=s@-DX rollout_sk.hip (the general
kernel's lane-skewed schedule; -DCCKA_SK_ONE instantiates <2, 8> only). Set VARIANTS_NO_MAKE=1 to link
against the objects already built.
usage: python tools/build_variants.py name=-DD1_S_V=3 [name2="-DA -DB" ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math", "-fPIC",
         "-Wall", "-Wno-unused-function"]
if not os.environ.get("VARIANTS_NO_MAKE"):
    subprocess.run(["make", "-s", "-C", CSRC], check=True)
procs = []
for arg in sys.argv[1:]:
    name, _, defs = arg.partition("=")
    src, base, extra = "rollout_d1.hip", "rollout_d1.o", []
    if defs.startswith("r@"):  # the general kernel's source (built with the MLP flags, as the Makefile does)
        defs, base, extra = defs[1:], "rollout.o", ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
    elif defs.startswith("p@"):  # the policy-gradient kernels' source
        defs, base, extra = defs[1:], "pg.o", ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
    elif defs.startswith("s@"):  # the lane-skewed general kernel's unit
        defs, src, base, extra = defs[2:], "rollout_sk.hip", "rollout_sk.o", ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
    elif defs.startswith("m@"):  # the MLP kernels' source
        defs, base, extra = defs[1:], "mlp.o", ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
    if defs.startswith("@"):  # NAME=@other.hip[:flags]: another source file in csrc/ (e.g. a committed version)
        src, _, defs = defs[1:].partition(":")
    out = os.path.join(CSRC, "build", "variants", name)
    os.makedirs(out, exist_ok=True)
    obj = os.path.join(out, base)
    procs.append((name, out, obj, subprocess.Popen(["/opt/rocm/bin/hipcc", *FLAGS, *extra, *defs.split(), "-c", "-o",
                                                    obj, os.path.join(CSRC, src)])))
for name, out, obj, p in procs:
    assert p.wait() == 0, name
    others = [os.path.join(CSRC, "build", f) for f in ("rollout.o", "rollout_multi.o", "rollout_pol.o", "rollout_sk.o",
                                                       "rollout_sk416.o", "rollout_d1.o", "rollout_pool.o", "sweep.o", "mlp.o", "pg.o",
                                                       "ccka_abi.o") if f != os.path.basename(obj)]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(out, "libccka.so"), obj, *others, "-L/opt/rocm/lib", "-lrccl",
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    print("built", name)
