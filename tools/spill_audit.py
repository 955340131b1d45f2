"""Where do a kernel's register spills sit?  Disassembles the gfx950 code object of a built object file and, per
kernel, counts the scratch (spill) instructions inside its innermost MFMA loop (the shortest backward-branch range
holding an MFMA) against its total:
  python tools/spill_audit.py camels-diffusion-model_amd/lib/gemm_f32.hip.o [name-substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def disassemble(obj: str) -> str:
    with tempfile.TemporaryDirectory() as td:
        fb, dev = os.path.join(td, "fb.bin"), os.path.join(td, "dev.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(td, "j.o")],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fb}", f"--output={dev}", "--unbundle"], check=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", dev], check=True,
                              capture_output=True, text=True).stdout


def kernels(text: str):
    cur, out = None, {}
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            cur = m.group(1)
            out[cur] = []
        elif cur and line.strip():
            out[cur].append(line.strip())
    return out


def audit(ins):
    addrs = []
    for x in ins:
        m = re.search(r"//\s*([0-9A-F]+):", x)
        addrs.append(int(m.group(1), 16) if m else None)
    a2i = {a: i for i, a in enumerate(addrs) if a is not None}
    loops = []
    for i, x in enumerate(ins):
        m = re.match(r"s_(cbranch_\w+|branch) (\d+)", x)
        if m and addrs[i] is not None:
            s = int(m.group(2))
            s = s - 65536 if s >= 32768 else s
            if s < 0 and (addrs[i] + 4 + 4 * s) in a2i:
                loops.append((a2i[addrs[i] + 4 + 4 * s], i))
    mf = [i for i, x in enumerate(ins) if "v_mfma" in x]
    sc = [i for i, x in enumerate(ins) if "scratch_" in x]
    inner = [(a, b) for a, b in loops if any(a <= k <= b for k in mf)]
    inner = min(inner, key=lambda t: t[1] - t[0]) if inner else None
    n_in = sum(1 for s in sc if inner and inner[0] <= s <= inner[1])
    return len(sc), n_in, inner


if __name__ == "__main__":
    obj, pats = sys.argv[1], sys.argv[2:]
    for name, ins in kernels(disassemble(obj)).items():
        if pats and not any(p in name for p in pats):
            continue
        total, n_in, inner = audit(ins)
        if total:
            d = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip().split("(")[0]
            print(f"{total:4d} spill ops, {n_in:3d} in the MFMA loop {inner}  {d}")
