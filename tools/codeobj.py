"""Fingerprint of one kernel's machine code in libgamesman_hip.so.

bench.py reports the PMC traffic of its dominant kernel from a committed
rocprofv3 --pmc summary (profiles/pmc_traffic.json) only while that summary
describes the code the bench runs.  Hashing whole source files made any edit
of those files -- a host-side default, a comment -- invalidate the figure
(VERDICT r4, weak 7); this hashes the bytes of the measured kernel's own
gfx950 functions instead: the offload bundle's gfx950 ELF, its symbol table,
the .text bytes of every symbol whose (mangled) name contains all the given
parts.

  python tools/codeobj.py gamesmanmpi_amd/libgamesman_hip.so k_plane_resolve_x2 ILi1ELi4ELb0E
"""
import hashlib
import struct
import sys

# kernel short name (as bench.py / pmc_summary.py key it) -> mangled-name
# parts of the instantiations the bench measures (8-bit words, 4 outer digits,
# one table)
MEASURED = {
    "k_plane_resolve_x2": ("k_plane_resolve_x2", "ILi1ELi4ELb0E"),
    "k_plane_run": ("k_plane_run", "ILi1ELi4ELb0ELb0E"),
    "k_rk_backward": ("k_rk_backward", "ILi6ELi4ELb0ELi0EE"),  # toot 6x4, one table, no A/B knob
    "k_rk_boards_sl": ("k_rk_boards_sl",),
    "k_rk_reach4": ("k_rk_reach4",),
}


def _gfx_elf(blob):
    i = blob.find(b"__CLANG_OFFLOAD_BUNDLE__")
    if i < 0:
        raise ValueError("no offload bundle")
    n = struct.unpack_from("<Q", blob, i + 24)[0]
    p = i + 32
    for _ in range(n):
        off, size, tl = struct.unpack_from("<QQQ", blob, p)
        p += 24
        triple = blob[p:p + tl].decode()
        p += tl
        if "gfx950" in triple and size:
            return blob[i + off:i + off + size]
    raise ValueError("no gfx950 code object")


def _symbols(elf):
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + k * shentsize) for k in range(shnum)]
    for sh in secs:
        if sh[1] != 2:  # SHT_SYMTAB
            continue
        strtab = secs[sh[6]]
        for k in range(sh[5] // sh[9]):
            name_off, info, other, shndx, value, size = struct.unpack_from("<IBBHQQ", elf, sh[4] + k * sh[9])
            if (info & 0xF) != 2 or not size or shndx >= len(secs):  # STT_FUNC
                continue
            end = elf.index(b"\0", strtab[4] + name_off)
            name = elf[strtab[4] + name_off:end].decode()
            sec = secs[shndx]
            yield name, elf[sec[4] + (value - sec[3]):sec[4] + (value - sec[3]) + size]


def kernel_code_sha16(so_path, kernel):
    """sha256[:16] over the code bytes of the measured instantiations of
    `kernel` (MEASURED), or None when the library or the symbols are missing."""
    parts = MEASURED.get(kernel, (kernel,))
    try:
        with open(so_path, "rb") as fh:
            elf = _gfx_elf(fh.read())
        h = hashlib.sha256()
        hit = 0
        for name, code in sorted(_symbols(elf)):
            if all(p in name for p in parts):
                h.update(name.encode())
                h.update(code)
                hit += 1
        return h.hexdigest()[:16] if hit else None
    except (OSError, ValueError, struct.error):
        return None


if __name__ == "__main__":
    print(kernel_code_sha16(sys.argv[1], sys.argv[2]))
