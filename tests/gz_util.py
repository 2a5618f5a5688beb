"""gzip / BGZF writers for the compressed-input tests (test_gzsrc.py, test_cli_gpu.py): members built
byte by byte (RFC 1952) so that every header shape a reader meets can be made -- BGZF 'BC' extra
subfields (SAM spec §4.1), FNAME / FCOMMENT / FHCRC / other FEXTRA fields, stored (level 0) members
whose payload holds a whole gzip file (false member starts inside the compressed stream)."""
import random
import struct
import zlib

BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def member(data, level=6, bgzf=False, fname=None, fcomment=None, fextra=None, fhcrc=False, bad_hcrc=False,
           bad_crc=False):
    """One gzip member of `data`."""
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    body = c.compress(data) + c.flush()
    flg = 0
    extra = b""
    if bgzf:
        flg |= 4
        extra = b"BC" + struct.pack("<H", 2) + b"\0\0"
    elif fextra is not None:
        flg |= 4
        extra = fextra
    if fname is not None:
        flg |= 8
    if fcomment is not None:
        flg |= 16
    if fhcrc:
        flg |= 2
    h = bytearray(b"\x1f\x8b\x08" + bytes([flg]) + b"\0\0\0\0\0\xff")
    if flg & 4:
        h += struct.pack("<H", len(extra)) + extra
    if fname is not None:
        h += fname + b"\0"
    if fcomment is not None:
        h += fcomment + b"\0"
    if fhcrc:
        hc = zlib.crc32(bytes(h)) & 0xFFFF
        h += struct.pack("<H", hc ^ (1 if bad_hcrc else 0))
    crc = zlib.crc32(data) & 0xFFFFFFFF
    if bad_crc:
        crc ^= 0x10
    out = bytes(h) + body + struct.pack("<II", crc, len(data) & 0xFFFFFFFF)
    if bgzf:
        bsize = len(out) - 1
        assert bsize <= 0xFFFF
        off = 12 + 4  # XLEN (2) at 10, subfield id/len at 12..15, BSIZE at 16
        out = out[:off] + struct.pack("<H", bsize) + out[off + 2:]
    return out


def bgzf(data, block=65280, level=6, eof=True):
    """BGZF: members of at most `block` input bytes, then the empty EOF member."""
    out = [member(data[i:i + block], level, bgzf=True) for i in range(0, len(data), block)]
    return b"".join(out) + (BGZF_EOF if eof else b"")


def multi(data, seed, lo=1, hi=300_000, level=6):
    """Plain gzip members of random input sizes (some empty), concatenated."""
    r = random.Random(seed)
    out, i = [], 0
    while i < len(data):
        k = r.randint(lo, hi)
        out.append(member(data[i:i + k], level))
        if r.random() < 0.05:
            out.append(member(b"", level))
        i += k
    return b"".join(out)


def fastq_text(n, seed, lmin=40, lmax=160):
    r = random.Random(seed)
    out = []
    for k in range(n):
        L = r.randint(lmin, lmax)
        s = "".join(r.choice("ACGT") for _ in range(L))
        q = "".join(r.choice("FFFFF:,#") for _ in range(L))
        out.append(f"@r{k} c{k}\n{s}\n+\n{q}\n")
    return "".join(out).encode()
