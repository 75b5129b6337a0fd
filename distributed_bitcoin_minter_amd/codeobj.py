"""Which machine code a search kernel is: the SHA-256 of its instruction
bytes inside the gfx950 code objects that libbtcminer.so embeds.

Each search-kernel object of the library carries its device code as a clang
offload bundle (`__CLANG_OFFLOAD_BUNDLE__`, csrc/Makefile: clang-offload-
bundler); the gfx950 entry of a bundle is an AMDGPU ELF whose symbol table
names every kernel.  The hash covers the kernel function's bytes in .text,
so two libraries give the same hash for a kernel exactly when its
instructions are identical -- what a PMC summary taken on one build needs to
be valid for another (tools/pmc_summary.py records it; bench.py compares it
with the library it loaded: roofline.pmc.same_kernel).

Pure file parsing: no GPU, no HIP call, no code executed from the file.
"""
import hashlib
import struct

_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def mangled_prefix(p, nbv=1, pad_block=0):
    """Itanium-mangled name prefix of the launch's kernel (bench.kernel_name):
    search_kernel<P, NBV>, search_kernel_padc<P, 1> (pad_block 2) or
    search_kernel_padk<P, K, 1> (pad_block 2 + K)."""
    if pad_block == 2:
        return f"_ZN2bm18search_kernel_padcILi{p}ELi1EEE"
    if pad_block > 2:
        return f"_ZN2bm18search_kernel_padkILi{p}ELi{pad_block - 2}ELi1EEE"
    return f"_ZN2bm13search_kernelILi{p}ELi{nbv}EEE"


def _bundles(data):
    """(triple, bytes) of every bundle entry in the file."""
    pos = data.find(_MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        off = pos + 32
        for _ in range(min(n, 64)):
            e_off, e_size, tlen = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24:off + 24 + tlen].decode("ascii", "replace")
            off += 24 + tlen
            if e_size:
                yield triple, data[pos + e_off:pos + e_off + e_size]
        pos = data.find(_MAGIC, pos + 24)


def _elf_functions(elf):
    """{symbol name: function bytes} of an ELF64 little-endian object."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        return {}
    e_shoff, = struct.unpack_from("<Q", elf, 0x28)
    e_shentsize, e_shnum, _ = struct.unpack_from("<HHH", elf, 0x3A)
    secs = []
    for i in range(e_shnum):
        name, typ, _flags, addr, off, size, link, _info, _al, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", elf, e_shoff + i * e_shentsize)
        secs.append((typ, addr, off, size, link, entsize))
    out = {}
    for typ, _addr, off, size, link, entsize in secs:
        if typ != 2 or not entsize:  # SHT_SYMTAB
            continue
        str_off = secs[link][2]
        for j in range(size // entsize):
            st_name, st_info, _other, st_shndx, st_value, st_size = struct.unpack_from(
                "<IBBHQQ", elf, off + j * entsize)
            if (st_info & 0xF) != 2 or not st_size or st_shndx >= len(secs):  # STT_FUNC
                continue
            end = elf.index(b"\0", str_off + st_name)
            name = elf[str_off + st_name:end].decode("ascii", "replace")
            _t, s_addr, s_off, _s, _l, _e = secs[st_shndx]
            start = s_off + (st_value - s_addr)
            out[name] = elf[start:start + st_size]
    return out


def kernel_code_sha(lib_path, p, nbv=1, pad_block=0, arch="gfx950"):
    """sha256 (hex) of the launch's kernel's instruction bytes in lib_path,
    or None when the library holds no such kernel (or cannot be read)."""
    try:
        data = open(lib_path, "rb").read()
    except OSError:
        return None
    want = mangled_prefix(p, nbv, pad_block)
    for triple, blob in _bundles(data):
        if arch not in triple:
            continue
        for name, code in _elf_functions(blob).items():
            if name.startswith(want):
                return hashlib.sha256(code).hexdigest()
    return None
