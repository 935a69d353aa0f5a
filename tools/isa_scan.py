"""Scan the gfx950 code objects inside a built libeosv.so for the store-data hazard found in r06.

A VMEM store of more than 64 bits (buffer_store_dwordx3/x4, global_store_dwordx3/x4) reads its data
VGPRs after issue; a VALU instruction that writes one of those VGPRs in the very next slot can land
before the store has read it.  The compiler pads that case only when the store's soffset is an
inline constant: with an SGPR soffset it assumes the hardware is safe, and on gfx950 it is not --
bneck_bf16_kernel<64,64,false> stored the lane LDS base of the following v_mov into one dword of
lanes 12/13 (tests/native/bneck_check.cpp).  The fused-block kernels store through
store_b128_guarded (common.h: an s_nop the scheduler cannot fill); the other kernels' schedules
have no such pair today, and this scan (tests/test_cpu_host.py) asserts that no store anywhere in
the library is directly followed by a VALU write of its data.

  python tools/isa_scan.py [<libeosv.so>]      -> prints every violation, exit 1 if any

Works on the uncompressed clang offload bundles hipcc -shared writes into .hip_fatbin."""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
WIDE_STORE = re.compile(r"^(buffer|global)_store_dwordx[34]\b")


def code_objects(lib):
    """[bytes] of every gfx950 ELF in the library's offload bundles."""
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fb.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fb}", lib,
                        os.path.join(td, "dummy")], check=True, capture_output=True)
        blob = open(fb, "rb").read()
    out = []
    pos = blob.find(MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", blob, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple:
                out.append(blob[pos + off:pos + off + size])
        pos = blob.find(MAGIC, pos + 1)
    return out


def _regs(text):
    s = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]", text):
        s.update(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", text):
        s.add(int(m.group(1)))
    return s


def disassemble(elf):
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "co.elf")
        open(p, "wb").write(elf)
        r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", "--no-leading-addr", p],
                           check=True, capture_output=True, text=True)
    return r.stdout


def violations(asm):
    """[(kernel, store, next instruction)] where a VALU writes a wide store's data VGPRs right after it."""
    out, fn, prev = [], "?", None
    for raw in asm.splitlines():
        line = raw.split(";")[0].strip()
        m = re.match(r"^([\w.$]+)>?:$", raw.strip().lstrip("<"))
        if m:
            fn, prev = m.group(1), None
            continue
        if not line:
            continue
        op = line.split()[0]
        if prev is not None and op.startswith("v_") and not op.startswith(("v_cmp_", "v_readfirstlane", "v_readlane")):
            dst = line.split(None, 1)[1].split(",")[0] if " " in line else ""
            if _regs(dst) & prev[1]:
                out.append((fn, prev[0], line))
        if WIDE_STORE.match(op):
            data = line.split(None, 1)[1].split(",")[1 if op.startswith("global") else 0]
            prev = (line, _regs(data))
        else:
            prev = None
    return out


def scan(lib):
    found = []
    for co in code_objects(lib):
        found += violations(disassemble(co))
    return found


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "embodied-one-shot-video-recognition_amd",
        "libeosv.so")
    found = scan(lib)
    for fn, st, nx in found:
        print(f"{fn}\n   {st}\n   {nx}")
    print(f"{len(found)} store-data hazards in {lib}")
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main())
