#!/usr/bin/env python
"""Static guard against the gfx950 store-data hazard hipcc 7.2 left unprotected (Kernels):
a packed f32 VALU instruction (v_pk_*) issued right after a wide vector-memory store (> 64-bit data:
dwordx3 / dwordx4 / b96 / b128) overwrote the store's data VGPRs before the store had read them,
with no wait state between them -- every second stored float came out wrong.

Scans the device code of every object under build/ (the .hip_fatbin section, unbundled for gfx950
and disassembled with ROCm's llvm-objdump) and reports each wide store followed, within the next
WINDOW instructions and with no s_nop between, by a v_pk_* whose destination overlaps the store's
data registers (the hazard needs one wait state: flagged when the v_pk_* is the very next
instruction; the store data of a 4-dword store is read a cycle after its issue).

    python tools/isa_hazard_check.py [build_dir]      (exit 1 on findings)

Second guard (--bitcast-lanes [src dirs]): ROCm 7.2's clang lowers `__builtin_bit_cast(T, v[i])`, with v an
ext_vector_type value and v[i] an element lvalue, to a load of the VECTOR's address: it returns element 0's
bits whatever i is (host and device alike; tools/bitcast_lane_probe.cpp shows it).  That was the round-4
"wrong dy" of the pooled-dz weight gradient (commit d4d63c9): the selection bytes held in lane 2 of the dz
vector were read back as `__builtin_bit_cast(unsigned, dzv[m][2])`, i.e. as the bits of the first pooled
gradient in lane 0 -- no FTZ or other float op touched them.  The guard flags every bit_cast whose operand is
a subscripted lvalue (`x[...]`); bit-cast a scalar temporary instead (`float t = v[i];`).
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
WINDOW = 1  # the hazard needs one wait state: any instruction in between provides it
STORE = re.compile(r"^\s*(buffer|global|flat|scratch)_store_(dwordx3|dwordx4|b96|b128)\b\s+(.*)$")
REG = re.compile(r"^v\[(\d+):(\d+)\]$|^v(\d+)$")


def regs(tok):
    tok = tok.strip().rstrip(",")
    m = REG.match(tok)
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def disassemble(obj, tmp):
    fat = os.path.join(tmp, "x.fatbin")
    co = os.path.join(tmp, "x.co")
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", obj], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}", "--unbundle"], check=True)
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True, text=True).stdout
    return out.splitlines()


def scan(lines):
    found = []
    insts = [ln.split("//")[0].rstrip() for ln in lines if ln.startswith("\t") or ln.startswith("  ")]
    insts = [i for i in insts if i.strip()]
    for k, ins in enumerate(insts):
        m = STORE.match(ins)
        if not m:
            continue
        ops = [o.strip() for o in m.group(3).split(",")]
        # data operand: buffer_store vdata, vaddr, ...; global / flat / scratch_store vaddr, vdata, ...
        data = regs(ops[0] if m.group(1) == "buffer" else ops[1] if len(ops) > 1 else "")
        for nxt in insts[k + 1:k + 1 + WINDOW]:
            op = nxt.split()[0]
            if op.startswith("s_nop") or op.startswith("s_waitcnt"):
                break
            if op.startswith("v_pk_"):
                dst = regs(nxt.split()[1])
                if dst & data:
                    found.append((ins.strip(), nxt.strip()))
    return found


# operand = a subscripted lvalue (v[i], v[m][2]) or a vector-lane accessor (v.x / .y / .z / .w, .r-.a, .s0-.sF,
# .hi / .lo / .even / .odd): both name an ext_vector_type element (tools/bitcast_lane_probe.cpp has each form)
BITCAST_SUB = re.compile(r"__builtin_bit_cast\s*\(\s*[^,()]+(?:\([^()]*\))?\s*,\s*("
                         r"[A-Za-z_][\w.]*\s*(?:\[[^\]]*\]\s*)+"
                         r"|[A-Za-z_][\w]*(?:\s*\[[^\]]*\])*(?:\.\w+)*\.(?:[xyzwrgba]|s[0-9a-fA-F]+|hi|lo|even|odd)\s*"
                         r")\)")


def scan_bitcast_lanes(dirs):
    """(file, line, text) of every __builtin_bit_cast whose operand is a subscripted lvalue or a vector-lane
    accessor."""
    found = []
    for d in dirs:
        for path in sorted(glob.glob(os.path.join(d, "*.hip")) + glob.glob(os.path.join(d, "*.h")) +
                           glob.glob(os.path.join(d, "*.cpp"))):
            if os.path.basename(path) == "bitcast_lane_probe.cpp":  # the defect's demonstration
                continue
            with open(path) as f:
                for n, line in enumerate(f, 1):
                    code = line.split("//")[0]
                    if BITCAST_SUB.search(code):
                        found.append((path, n, line.strip()))
    return found


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--bitcast-lanes":
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        dirs = sys.argv[2:] or [os.path.join(root, "phoneme_contrast_amd", "csrc"), os.path.join(root, "tools")]
        bad = scan_bitcast_lanes(dirs)
        for path, n, text in bad:
            print(f"{os.path.relpath(path)}:{n}: bit_cast of a vector-element lvalue: {text}")
        print(f"{len(bad)} bit_cast lane finding(s)")
        return 1 if bad else 0
    bdir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "build")
    objs = sorted(glob.glob(os.path.join(bdir, "*.o")))
    if not objs:
        print(f"no objects under {bdir}")
        return 2
    bad = 0
    with tempfile.TemporaryDirectory() as tmp:
        for o in objs:
            for st, pk in scan(disassemble(o, tmp)):
                print(f"{os.path.basename(o)}: {st}  ->  {pk}")
                bad += 1
    print(f"{len(objs)} objects scanned, {bad} hazard(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
