"""Compare the device compressor's dumped frames (tools/zstd_write_probe.py)
with the oracle's, section by section: frame header, block header, literals
section (header, tree description, jump table, streams), sequences header,
table descriptions, bitstream. Debugging aid (CPU only).

    python tools/zstd_write_diff.py DIR [level]
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
from oracle import zstd_encoder as ze  # noqa: E402
from oracle import zstd_oracle as zo  # noqa: E402


def sections(f: bytes):
    """[(name, bytes)] of a one-block frame."""
    out = []
    h = zo.frame_header(f)
    out.append(("frame", f[:h.size]))
    q = h.size
    bh = int.from_bytes(f[q:q + 3], "little")
    out.append(("block_hdr", f[q:q + 3]))
    q += 3
    bt, bs = (bh >> 1) & 3, bh >> 3
    if bt != 2:
        out.append(("block_body", f[q:]))
        return out
    end = q + bs
    b0 = f[q]
    lt, sf = b0 & 3, (b0 >> 2) & 3
    if lt in (0, 1):
        if sf in (0, 2):
            n, hs = b0 >> 3, 1
        elif sf == 1:
            n, hs = (b0 >> 4) + (f[q + 1] << 4), 2
        else:
            n, hs = (b0 >> 4) + (f[q + 1] << 4) + (f[q + 2] << 12), 3
        ln = n if lt == 0 else 1
        out.append((f"lit_hdr(type {lt})", f[q:q + hs]))
        out.append(("lit_body", f[q + hs:q + hs + ln]))
        q += hs + ln
    else:
        hs = [3, 3, 4, 5][sf]
        hv = int.from_bytes(f[q:q + hs], "little")
        bits = [10, 10, 14, 18][sf]
        csize = (hv >> (4 + bits)) & ((1 << bits) - 1)
        out.append((f"lit_hdr(type {lt} sf {sf})", f[q:q + hs]))
        p = q + hs
        tb = f[p]
        tl = 1 + (tb if tb < 128 else (tb - 127 + 1) // 2)
        out.append(("huf_tree", f[p:p + tl]))
        p2 = p + tl
        if sf != 0:
            out.append(("jump", f[p2:p2 + 6]))
            s1 = int.from_bytes(f[p2:p2 + 2], "little")
            s2 = int.from_bytes(f[p2 + 2:p2 + 4], "little")
            s3 = int.from_bytes(f[p2 + 4:p2 + 6], "little")
            a = p2 + 6
            out += [("stream1", f[a:a + s1]), ("stream2", f[a + s1:a + s1 + s2]),
                    ("stream3", f[a + s1 + s2:a + s1 + s2 + s3]),
                    ("stream4", f[a + s1 + s2 + s3:q + hs + csize])]
        else:
            out.append(("stream", f[p2:q + hs + csize]))
        q += hs + csize
    b0 = f[q]
    if b0 < 128:
        ns, c = b0, 1
    elif b0 < 255:
        ns, c = ((b0 - 128) << 8) + f[q + 1], 2
    else:
        ns, c = f[q + 1] + (f[q + 2] << 8) + 0x7F00, 3
    out.append(("nseq", f[q:q + c]))
    q += c
    if ns:
        out.append(("modes", f[q:q + 1]))
        out.append(("tables+bits", f[q + 1:end]))
    return out


def main():
    d = Path(sys.argv[1])
    level = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    spec = json.loads((d / f"zw_{level}.json").read_text())
    ib = (d / f"zw_inputs_{level}.bin").read_bytes()
    fb = (d / f"zw_frames_{level}.bin").read_bytes()
    ins, frs, p, q = [], [], 0, 0
    for n, m in zip(spec["inputs"], spec["frames"]):
        ins.append(ib[p:p + n])
        frs.append(fb[q:q + m])
        p += n
        q += m
    bad = 0
    for k, (x, g) in enumerate(zip(ins, frs)):
        want = ze.compress(x, level)
        if g == want:
            continue
        bad += 1
        if bad > 12:
            continue
        try:
            ok = zo.decompress(g, len(x)) == x
        except zo.Corrupt as e:
            ok = f"corrupt: {e}"
        print(f"--- input {k} n={len(x)} status={spec['status'][k]} dev {len(g)} oracle "
              f"{len(want)} decodes={ok}")
        sg, sw = sections(g), sections(want)
        for (na, va), (nb, vb) in zip(sg, sw):
            flag = "" if (na == nb and va == vb) else "   <== DIFF"
            print(f"  {na:24s} {len(va):5d} | {nb:24s} {len(vb):5d}{flag}")
            if flag and len(va) < 40:
                print("     dev", va.hex(), "\n     orc", vb.hex())
    print("mismatches", bad, "of", len(ins))


if __name__ == "__main__":
    main()
