#!/usr/bin/env python3
"""Static decode of the CMSIS-DSP routines behind arm_rfft_q31 in the
reference's prebuilt evb/libs/libCMSISDSP.a -- read as bytes, never executed.

Test infrastructure: the CMSIS source is not vendored, so
the oracle's restatement of the fixed-point rFFT (oracle/nnsp_oracle.c:29-170)
is pinned to the shipped binary only through its tables.  This tool walks the
Thumb-2 instruction stream of the functions the restatement follows and
counts the multiply forms (SMMUL = truncating high word, SMMULR / SMMLAR /
SMMLSR = rounded, SMULL / SMLAL = full 64-bit) and the immediate shift
amounts, so that the restatement's arithmetic choices -- truncating products
in the radix-4 butterflies, rounded ones in the split, the guard-bit shifts
(>> 4 in, << 1 / >> 1 / >> 2 per stage) -- are checked against the shipped code.

usage: cmsis_decode.py [ARCHIVE] > tests/golden/cmsis_decode.json
The JSON it writes is data (instruction counts), committed as a fixture.
"""
import json
import struct
import sys

FUNCS = {
    "arm_cfft_radix4_q31.c.obj": ["arm_radix4_butterfly_q31", "arm_radix4_butterfly_inverse_q31", "arm_cfft_radix4_q31"],
    "arm_cfft_q31.c.obj": ["arm_cfft_q31", "arm_cfft_radix4by2_q31", "arm_cfft_radix4by2_inverse_q31"],
    "arm_rfft_q31.c.obj": ["arm_rfft_q31", "arm_split_rfft_q31", "arm_split_rifft_q31"],
    "arm_bitreversal2.c.obj": ["arm_bitreversal_32"],
}


def ar_members(data):
    """(name, bytes) of a System V / GNU ar archive."""
    assert data[:8] == b"!<arch>\n", "not an ar archive"
    off, longnames, out = 8, b"", {}
    while off + 60 <= len(data):
        h = data[off:off + 60]
        name = h[:16].decode().strip()
        size = int(h[48:58])
        body = data[off + 60:off + 60 + size]
        if name == "//":
            longnames = body
        elif name.startswith("/") and name[1:].isdigit():
            i = int(name[1:])
            out[longnames[i:longnames.index(b"/\n", i)].decode()] = body
        elif name not in ("/", ""):
            out[name.rstrip("/")] = body
        off += 60 + size + (size & 1)
    return out


def elf_functions(obj):
    """{function name: bytes of its code} of an ELF32 little-endian ARM object."""
    assert obj[:4] == b"\x7fELF" and obj[4] == 1 and obj[5] == 1, "not ELF32 LE"
    e_shoff, = struct.unpack_from("<I", obj, 0x20)
    e_shentsize, e_shnum, e_shstrndx = struct.unpack_from("<HHH", obj, 0x2E)
    secs = [struct.unpack_from("<IIIIIIIIII", obj, e_shoff + i * e_shentsize) for i in range(e_shnum)]
    # (name, type, flags, addr, offset, size, link, info, addralign, entsize)
    symtab = next(s for s in secs if s[1] == 2)
    strtab = secs[symtab[6]]
    out = {}
    for i in range(symtab[5] // 16):
        st_name, st_value, st_size, st_info, _, st_shndx = struct.unpack_from("<IIIBBH", obj, symtab[4] + 16 * i)
        if st_info & 0xF != 2 or st_shndx == 0 or st_shndx >= e_shnum:   # STT_FUNC, defined
            continue
        end = obj.index(b"\0", strtab[4] + st_name)
        name = obj[strtab[4] + st_name:end].decode()
        sec = secs[st_shndx]
        start = sec[4] + (st_value & ~1)   # Thumb bit
        out[name] = obj[start:start + st_size]
    return out


def decode(code):
    """Counts of multiply forms and immediate shifts in a Thumb-2 stream."""
    c = {"insns": 0, "smmul": 0, "smmulr": 0, "smmla": 0, "smmlar": 0, "smmls": 0, "smmlsr": 0,
         "smull": 0, "smlal": 0, "mul32": 0, "adc": 0, "sbc": 0, "imm_2p31": 0, "shifts": {}}

    def shift(kind, n):
        k = f"{kind}#{n}"
        c["shifts"][k] = c["shifts"].get(k, 0) + 1

    i = 0
    while i + 2 <= len(code):
        h1, = struct.unpack_from("<H", code, i)
        c["insns"] += 1
        if (h1 >> 11) in (0b11101, 0b11110, 0b11111) and i + 4 <= len(code):
            h2, = struct.unpack_from("<H", code, i + 2)
            i += 4
            op = h1 >> 4
            ra, r = h2 >> 12, (h2 >> 4) & 1
            if op == 0xFB5 and (h2 >> 5) & 7 == 0:          # SMMUL{R} (Ra = 15) / SMMLA{R}
                c[("smmul" if ra == 15 else "smmla") + ("r" if r else "")] += 1
            elif op == 0xFB6 and (h2 >> 5) & 7 == 0:        # SMMLS{R}
                c["smmls" + ("r" if r else "")] += 1
            elif op == 0xFB8 and (h2 >> 4) & 0xF == 0:      # SMULL
                c["smull"] += 1
            elif op == 0xFBC and (h2 >> 4) & 0xF == 0:      # SMLAL
                c["smlal"] += 1
            elif op == 0xFB0 and (h2 >> 4) & 0xF == 0:      # MUL / MLA
                c["mul32"] += 1
            elif (h1 & 0xFBE0) == 0xF140 or (h1 & 0xFFE0) == 0xEB40:   # ADC{S}.W imm / reg
                c["adc"] += 1
            elif (h1 & 0xFBE0) == 0xF160 or (h1 & 0xFFE0) == 0xEB60:   # SBC{S}.W imm / reg
                c["sbc"] += 1
            elif ((h1 & 0xFBE0) in (0xF100, 0xF040) and (h1 & 0xFBEF) != 0xF10D) and not (h2 & 0x8000):
                # ADD{S}.W / MOV{S}.W (modified immediate): 0x400 expands to 0x80000000,
                # the rounding constant of the SMMULR / SMMLAR / SMMLSR forms
                imm12 = ((h1 >> 10) & 1) << 11 | ((h2 >> 12) & 7) << 8 | (h2 & 0xFF)
                if imm12 == 0x400:
                    c["imm_2p31"] += 1
            elif (h1 & 0xFFEF) == 0xEA4F or (h1 >> 9) == 0b1110101 and (h1 >> 5) & 0xF in (0b0000, 0b1000, 0b1101):
                # MOV.W / ADD.W / SUB.W (register, shifted): imm3:imm2, type
                amt = ((h2 >> 12) & 7) << 2 | (h2 >> 6) & 3
                typ = (h2 >> 4) & 3
                if amt or typ:
                    shift(("lsl", "lsr", "asr", "ror")[typ], amt if amt or typ == 0 else 32)
        else:
            i += 2
            if (h1 & 0xFFC0) == 0x4140:                      # ADCS (16-bit)
                c["adc"] += 1
            elif (h1 & 0xFFC0) == 0x4180:                    # SBCS (16-bit)
                c["sbc"] += 1
            elif (h1 >> 11) == 0b00010:                      # ASRS Rd, Rm, #imm5
                shift("asr", ((h1 >> 6) & 31) or 32)
            elif (h1 >> 11) == 0b00000 and (h1 >> 6) & 31:   # LSLS Rd, Rm, #imm5
                shift("lsl", (h1 >> 6) & 31)
            elif (h1 >> 11) == 0b00001:                      # LSRS
                shift("lsr", ((h1 >> 6) & 31) or 32)
    return c


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/evb/libs/libCMSISDSP.a"
    members = ar_members(open(path, "rb").read())
    out = {"archive": path.split("/root/reference/")[-1], "functions": {}}
    for obj, names in FUNCS.items():
        funcs = elf_functions(members[obj])
        for n in names:
            if n in funcs:
                d = decode(funcs[n])
                d["bytes"] = len(funcs[n])
                d["object"] = obj
                out["functions"][n] = d
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
