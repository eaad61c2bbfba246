"""Generate nem-mcmc-optimization_amd/csrc/refmath_tables.h: the data the
bit-exact restatements in refmath.h need, read from the libraries the
reference's arithmetic runs in (this container's, which are also the GPU
box host's: tools/host_blas_probe.py gives the same hashes on both):

* glibc 2.35 libm ``__exp_data.tab`` (exp, 128-entry 2^(i/128) table as
  (tail, scale-bits) pairs), located by its ``invln2N`` field;
* numpy 2.2.6 ``_multiarray_umath`` ``__svml_dlog_ha_data_internal_avx512``
  (16-entry -log(r) table, hi and lo parts) and
  ``__svml_dexp_ha_data_internal_avx512`` (16-entry 2^(j/16) table, hi and
  lo parts), at the addresses the code of ``__svml_log8_ha`` /
  ``__svml_exp8_ha`` loads them from (found with objdump, below);
* the 16 switch points of RNE_{1/32}(vrcp14pd(m)) over m in [1, 2), the
  reduction point of ``__svml_log8_ha``: vrcp14pd reads only the top 22
  mantissa bits and the rounded value is monotone in them, so the step
  function is exactly these thresholds (measured on this CPU with the
  instruction itself by a small AVX-512 program).

    python tools/gen_refmath_tables.py    (build container only)
"""
import os
import re
import struct
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "nem-mcmc-optimization_amd", "csrc", "refmath_tables.h")
LIBM = "/lib/x86_64-linux-gnu/libm.so.6"


def numpy_umath():
    import numpy._core._multiarray_umath as m
    return m.__file__


def symbol_addr(lib, name):
    out = subprocess.run(["nm", "-D", lib], capture_output=True, text=True, check=True).stdout
    for line in out.splitlines():
        p = line.split()
        if len(p) == 3 and p[2] == name:
            return int(p[0], 16)
    raise KeyError(name)


def data_block(lib, func):
    """The rodata block __svml_*_data_internal_avx512 a SVML entry point loads."""
    a = symbol_addr(lib, func)
    dis = subprocess.run(["objdump", "-d", "--no-show-raw-insn", lib, f"--start-address={a:#x}",
                          f"--stop-address={a + 0x200:#x}"], capture_output=True, text=True, check=True).stdout
    m = re.search(r"# ([0-9a-f]+) <(__svml_d\w+_data_internal_avx512)>", dis)
    if m:
        return int(m.group(1), 16)
    m = re.search(r"# ([0-9a-f]+) <(__svml_d\w+_data_internal_avx512)\+0x([0-9a-f]+)>", dis)
    return int(m.group(1), 16) - int(m.group(3), 16)


def vaddr_to_offset(lib, vaddr):
    out = subprocess.run(["readelf", "-lW", lib], capture_output=True, text=True, check=True).stdout
    for line in out.splitlines():
        p = line.split()
        if p and p[0] == "LOAD":
            off, va, fsz = int(p[1], 16), int(p[2], 16), int(p[4], 16)
            if va <= vaddr < va + fsz:
                return vaddr - va + off
    raise ValueError(hex(vaddr))


RCP_C = r"""
#include <immintrin.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
int main(void) {
  double prev = 2.0;
  for (uint64_t p = 0; p < (1ull << 22); p += 8) {
    double m[8], o[8];
    for (int l = 0; l < 8; l++) { uint64_t u = 0x3ff0000000000000ull | ((p + l) << 30); memcpy(&m[l], &u, 8); }
    _mm512_storeu_pd(o, _mm512_roundscale_pd(_mm512_rcp14_pd(_mm512_loadu_pd(m)), 0x58));
    for (int l = 0; l < 8; l++) {
      if (o[l] > prev) { printf("NONMONOTONE\n"); return 1; }
      if (o[l] != prev && p + l > 0) printf("%llu %.17g\n", (unsigned long long)(p + l), o[l]);
      prev = o[l];
    }
  }
  return 0;
}
"""


def rcp14_thresholds():
    with tempfile.TemporaryDirectory() as td:
        src, exe = os.path.join(td, "r.c"), os.path.join(td, "r")
        open(src, "w").write(RCP_C)
        subprocess.run(["gcc", "-O2", "-mavx512f", "-o", exe, src], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    th = [int(line.split()[0]) for line in out if line.strip()]
    vals = [float(line.split()[1]) for line in out if line.strip()]
    assert len(th) == 16 and vals == [(31 - k) / 32 for k in range(16)], (th, vals)
    return th


def fmt(vals, per=4):
    rows = []
    for k in range(0, len(vals), per):
        rows.append("    " + ", ".join(f"0x{v:016x}ull" for v in vals[k:k + per]) + ",")
    return "\n".join(rows)


def main():
    libm = open(LIBM, "rb").read()
    key = struct.pack("<d", float.fromhex("0x1.71547652b82fep0") * 128)
    assert libm.count(key) == 1
    i = libm.find(key)
    head = struct.unpack("<8d", libm[i:i + 64])
    assert head[1] == float.fromhex("0x1.8p52") and head[2] == float.fromhex("-0x1.62e42fefa0000p-8")
    exptab = struct.unpack("<256Q", libm[i + 112:i + 112 + 2048])
    lib = numpy_umath()
    raw = open(lib, "rb").read()

    def lanes(base, off):
        o = vaddr_to_offset(lib, base + off)
        return struct.unpack("<8Q", raw[o:o + 64])

    lg = data_block(lib, "__svml_log8_ha")
    ex = data_block(lib, "__svml_exp8_ha")
    loghi, loglo = lanes(lg, 0) + lanes(lg, 0x40), lanes(lg, 0x80) + lanes(lg, 0xc0)
    exphi, explo = lanes(ex, 0) + lanes(ex, 0x40), lanes(ex, 0x80) + lanes(ex, 0xc0)
    th = rcp14_thresholds()
    # the same step function by 64 buckets of the 22-bit prefix (p >> 16):
    # the thresholds are more than 2^16 apart, so a bucket holds at most one
    assert all(b - a > (1 << 16) for a, b in zip(th, th[1:])) and th[0] > 0
    base = [sum(1 for t in th if t < (bk << 16)) for bk in range(64)]
    inb = [next((t for t in th if (t >> 16) == bk), 0xFFFFFFFF) for bk in range(64)]
    for p in range(0, 1 << 22, 977):   # spot check here; tests check every prefix
        assert base[p >> 16] + (p >= inb[p >> 16]) == sum(1 for t in th if p >= t)
    import numpy
    text = f"""// GENERATED by tools/gen_refmath_tables.py -- do not edit.
// Data of the libraries the reference's arithmetic runs in (glibc 2.35 libm,
// numpy {numpy.__version__} SVML), for the bit-exact restatements in refmath.h.
// Origins and licences: glibc's exp table (LGPL-2.1-or-later; exp by Arm),
// Intel SVML's tables as bundled in numpy (BSD-3-Clause) -- THIRD_PARTY_NOTICES.md.
#pragma once
#include <stdint.h>

namespace nemo {{
namespace refmath {{

// glibc __exp_data.tab: [2 i] = bits of the tail of 2^(i/128), [2 i + 1] =
// bits of 2^(i/128) minus i << 45
constexpr uint64_t kGlibcExpTab[256] = {{
{fmt(exptab)}
}};

// __svml_log8_ha: -log(r) (r < 0.75: -log(2 r)) for r = 0.5 (1 + j/16) / 1,
// hi and lo parts, indexed by the top 4 mantissa bits of r
constexpr uint64_t kSvmlLogHi[16] = {{
{fmt(loghi)}
}};
constexpr uint64_t kSvmlLogLo[16] = {{
{fmt(loglo)}
}};

// __svml_exp8_ha: 2^(j/16), hi and lo parts
constexpr uint64_t kSvmlExpHi[16] = {{
{fmt(exphi)}
}};
constexpr uint64_t kSvmlExpLo[16] = {{
{fmt(explo)}
}};

// RNE_{{1/32}}(vrcp14pd(m)) for m in [1, 2) is (32 - n) / 32, n = the number of
// these thresholds <= the top 22 mantissa bits of m (measured on the
// instruction; monotone)
constexpr uint32_t kRcp14Switch[16] = {{
    {", ".join(str(v) for v in th)}
}};
// ... and by bucket p >> 16: n = kRcp14Base[b] + (p >= kRcp14InBucket[b])
constexpr uint32_t kRcp14Base[64] = {{
    {", ".join(str(v) for v in base)}
}};
constexpr uint32_t kRcp14InBucket[64] = {{
    {", ".join(f"0x{v:x}u" for v in inb)}
}};

}}  // namespace refmath
}}  // namespace nemo
"""
    open(OUT, "w").write(text)
    print("wrote", os.path.normpath(OUT))


if __name__ == "__main__":
    main()
