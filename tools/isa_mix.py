"""Static VALU instruction-class histogram of every kernel in the built library, and the kernel's
mix-weighted VALU issue roof from the measured per-class rates (tools/valu_rates.hip,
profiles/r5d_valu_rates.txt).

The roof: a kernel whose VALU instructions are the fractions f_c of classes with sustained rates
r_c (fraction of the nominal one-wave64-instruction-per-2-cycles issue) can at best issue at
1 / sum_c(f_c / r_c) of nominal -- the harmonic mean a stream of that mix sustains when nothing
else stalls it. `bench.py` divides a kernel's measured VALU issue rate (SQ_INSTS_VALU per dispatch
/ dispatch time) by that roof: the kernel's VALU fraction of its own mix peak.

The histogram is static (each instruction of the kernel's code once): the hot loops of the
front-end kernels are fully unrolled or dominate their bodies, so the static mix stands for the
dynamic one; SQ_INSTS_VALU (dynamic) carries the count. The rate column is the one for the
kernel's occupancy (waves per SIMD from its VGPR / AGPR / LDS use, w1/w2/w4/w8).

The code objects come straight out of the library: the .hip_fatbin section holds one clang
offload bundle per translation unit; the gfx950 entries are disassembled with llvm-objdump.
Usage: python tools/isa_mix.py [lib.so] > profiles/isa_mix.json"""
import collections
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# mnemonic (without the _e32/_e64/_sdwa/_dpp suffix) -> measured class of r5d_valu_rates.txt
CLASS_OF = [
    (r"v_(add|sub|subrev)_(u32|co_u32|i32|nc_u32|co_ci_u32|nc_i32)$", "add_u32"),
    (r"v_(xor|or)_b32$", "xor_b32"),
    (r"v_and_b32$", "and_b32"),
    (r"v_(lshrrev|lshlrev|ashrrev)_b32$", "lshrrev"),
    (r"v_(xor3|or3|and_or|xad_u32|bitop3)_b\d+$|v_bitop3", "bitop3"),
    (r"v_mul_lo_u32$|v_mul_hi_u32$|v_mad_u64_u32$|v_mul_lo_i32$", "mul_lo_u32"),
    (r"v_mul_(u32_u24|i32_i24)$", "mul_u32_u24"),
    (r"v_mul_hi_(u32_u24|i32_i24)$", "mul_hi_u24"),
    (r"v_mad_(u32_u24|i32_i24)$", "mad_u32_u24"),
    (r"v_(lshl_add|add_lshl|lshl_or|and_or|add3|sub3)_u32$|v_lshl_add_u64$", "add3"),
    (r"v_bfe_[ui]32$|v_bfi_b32$|v_bfm_b32$", "bfe_u32"),
    (r"v_(min|max|min3|max3|med3)_[ui]32$|v_(min3|max3|med3)_u32$", "min_u32"),
    (r"v_cndmask_b32$", "cndmask_s"),
    (r"v_(dot4|dot2|dot8)\w*", "udot4"),
    (r"v_alignbit_b32$", "alignbit"),
    (r"v_alignbyte_b32$", "alignbyte"),
    (r"v_perm_b32$", "perm"),
    (r"v_lerp_u8$", "lerp_u8"),
    (r"v_(sad|msad|qsad|mqsad)_\w+$", "sad_u8"),
    (r"v_pk_(add|sub)_[ui]16$", "pk_add_u16"),
    (r"v_pk_(min|max)_[ui]16$", "pk_min_i16"),
    (r"v_pk_(mad|mul_lo)_[ui]16$|v_pk_lshl\w*|v_pk_lshr\w*|v_pk_ashr\w*", "pk_mad_i16"),
    (r"v_pk_(add|mul|fma)_f(16|32)$", "pk_add_f16"),
    (r"v_pk_(min|max)\w*_f16$", "pk_min_f16"),
    (r"v_pk_minimum3_f16$|v_pk_maximum3_f16$", "pk_minimum3_f16"),
    (r"v_(add|sub|subrev)_f32$", "add_f32"),
    (r"v_mul_f32$|v_mul_legacy_f32$", "mul_f32"),
    (r"v_(fma|fmac|mac|mad|fmaak|fmamk)_f32$", "fma_f32"),
    (r"v_cvt_\w+$|v_frexp\w*|v_ldexp\w*", "cvt_f32_u32"),
]
# classes the probe did not time: full-rate (VOP2/VOP1 moves, compares, f32 min/max) or the
# VOP3 integer rate (everything else)
FULL_RATE = re.compile(r"v_(mov|cmp|cmpx|readfirstlane|min_f32|max_f32|not_b32|bcnt|ffbh|ffbl"
                       r"|bfrev|mov_b64|swap|nop|mbcnt|readlane|writelane|accvgpr)\w*")
NON_VALU = re.compile(r"v_mfma\w*|v_smfmac\w*")
TRANS = re.compile(r"v_(rcp|rsq|sqrt|exp|log|sin|cos)_\w+")


def load_rates(path):
    rates = {}
    for line in open(path):
        m = re.match(r"(\S+)\s+w1 ([\d.]+)\s+w2 ([\d.]+)\s+w4 ([\d.]+)\s+w8 ([\d.]+)", line)
        if m:
            rates[m.group(1)] = {1: float(m.group(2)), 2: float(m.group(3)), 4: float(m.group(4)),
                                 8: float(m.group(5))}
    return rates


def code_objects(lib):
    """gfx950 code objects of every offload bundle in lib's .hip_fatbin section."""
    out = subprocess.run([READELF, "-S", "-W", lib], capture_output=True, text=True, check=True).stdout
    m = re.search(r"\.hip_fatbin\s+\S+\s+([0-9a-f]+)\s+([0-9a-f]+)\s+([0-9a-f]+)", out)
    if not m:
        raise SystemExit(f"{lib}: no .hip_fatbin section")
    off, size = int(m.group(2), 16), int(m.group(3), 16)
    with open(lib, "rb") as f:
        f.seek(off)
        blob = f.read(size)
    objs = []
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and esize:
                objs.append(blob[pos + eoff:pos + eoff + esize])
        pos = blob.find(MAGIC, pos + 32)
    return objs


def kernel_meta(co_path):
    """kernel symbol -> (vgprs + agprs, lds bytes) from the code object's notes."""
    out = subprocess.run([READELF, "--notes", "-W", co_path], capture_output=True, text=True).stdout
    meta = {}
    for blk in out.split(".name:")[1:]:
        name = blk.split("\n")[0].strip()
        g = lambda key: int((re.search(r"\.%s:\s+(\d+)" % key, blk) or [0, 0])[1])
        meta[name] = (g("vgpr_count") + g("agpr_count"), g("group_segment_fixed_size"))
    return meta


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names),
                         capture_output=True, text=True).stdout.split("\n")
    return {n: d.replace("slamgpu::", "").replace("(anonymous namespace)::", "").split("(")[0]
            .replace("void ", "") for n, d in zip(names, out)}


def occupancy(vgprs, lds, wg_waves=4):
    """waves per SIMD: 512 registers per lane (VGPR + AGPR, granule 8) and 160 KB of LDS per CU"""
    w = 8
    if vgprs:
        w = min(w, 512 // (-(-vgprs // 8) * 8))
    if lds:
        w = min(w, max(1, (160 * 1024 // lds) * wg_waves // 4))
    return max(1, w)


def classify(mn):
    mn = re.sub(r"_(e32|e64|sdwa|dpp)$", "", mn)
    if NON_VALU.fullmatch(mn):
        return None
    for pat, cls in CLASS_OF:
        if re.fullmatch(pat, mn):
            return cls
    if FULL_RATE.fullmatch(mn):
        return "add_u32"       # full-rate VOP1/VOP2-class issue
    if TRANS.fullmatch(mn):
        return "trans"
    return "other_vop3"


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "slam_framework_amd",
                                                             "libslamgpu.so")
    rates = load_rates(os.path.join(ROOT, "profiles", "r5d_valu_rates.txt"))
    # untimed classes: transcendental ops issue at a quarter rate; other VOP3 integer ops as the
    # measured VOP3 integer classes (mad_u32_u24)
    rates["trans"] = {w: 0.25 * rates["mul_f32"][w] for w in (1, 2, 4, 8)}
    rates["other_vop3"] = rates["mad_u32_u24"]
    kernels = {}
    with tempfile.TemporaryDirectory() as td:
        for i, co in enumerate(code_objects(lib)):
            p = os.path.join(td, f"co{i}.o")
            with open(p, "wb") as f:
                f.write(co)
            meta = kernel_meta(p)
            dis = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", p], capture_output=True,
                                 text=True, check=True).stdout
            cur, hist = None, None
            for line in dis.split("\n"):
                m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
                if m:
                    cur = m.group(1)
                    hist = None if cur.endswith(".kd") or cur not in meta else \
                        kernels.setdefault(cur, {"hist": collections.Counter(), "meta": meta[cur]})
                    continue
                if hist is None:
                    continue
                t = line.strip().split()
                if t and t[0].startswith("v_"):
                    c = classify(t[0])
                    if c:
                        hist["hist"][c] += 1
    names = demangle(list(kernels))
    res = {"source": "tools/isa_mix.py: static VALU class histogram of each kernel in "
                     "libslamgpu.so x the per-class sustained rates of profiles/r5d_valu_rates.txt "
                     "at the kernel's occupancy; roof = 1 / sum(f_c / r_c) of the nominal "
                     "1.2288e12 wave-instr/s", "kernels": {}}
    for sym, k in kernels.items():
        tot = sum(k["hist"].values())
        if not tot:
            continue
        w = occupancy(*k["meta"])
        col = max(c for c in (1, 2, 4, 8) if c <= w)
        inv = sum(n / tot / rates[c][col] for c, n in k["hist"].items())
        res["kernels"][names[sym]] = {
            "valu_static_instr": tot, "waves_per_simd": w, "rate_column": f"w{col}",
            "mix_roof_frac_of_nominal": round(1.0 / inv, 4),
            "classes": {c: round(n / tot, 4) for c, n in k["hist"].most_common()}}
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
