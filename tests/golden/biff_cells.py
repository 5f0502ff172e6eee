"""A second, separately written reader of the reference's demo/demodata.xls --
test infrastructure, written from the file formats, not from vbhem_amd/xls.py,
so that the committed fixture (tests/golden/demo_fixations.npz) does not come
from the reader it checks.

Scope is the minimum the demo file needs:
  * the OLE2 compound-file container: header, FAT (DIFAT in the header and in
    chained DIFAT sectors), directory, the "Workbook" stream (regular or mini
    stream);
  * BIFF8 records of the first worksheet: shared strings (SST + CONTINUE, with
    the high-byte flag restated at every CONTINUE boundary), LABELSST, NUMBER,
    RK and MULRK cells;
  * the row loop of src/util/read_xls_fixations.m:84-138 (subjects and trials in
    order of first appearance, numeric ids printed with %g, FixD optional).
"""
import struct

import numpy as np


# --------------------------------------------------------------------------
# compound file
# --------------------------------------------------------------------------
def _stream(blob: bytes, want=("Workbook", "Book")) -> bytes:
    if blob[:8] != bytes.fromhex("D0CF11E0A1B11AE1"):
        raise ValueError("not a compound file")
    ssz = 1 << struct.unpack_from("<H", blob, 0x1E)[0]
    msz = 1 << struct.unpack_from("<H", blob, 0x20)[0]
    n_fat, dir0 = struct.unpack_from("<II", blob, 0x2C)
    cutoff, mfat0, n_mfat, difat0, n_difat = struct.unpack_from("<IIIII", blob, 0x38)

    def sector(k):
        off = (k + 1) * ssz
        return blob[off:off + ssz]

    per = ssz // 4
    fat_secs = list(struct.unpack_from("<109I", blob, 0x4C))
    k = difat0
    for _ in range(n_difat):
        ids = struct.unpack(f"<{per}I", sector(k))
        fat_secs += ids[:-1]
        k = ids[-1]
    fat = []
    for k in fat_secs[:n_fat]:
        fat += struct.unpack(f"<{per}I", sector(k))

    def chain(start, table):
        out, k = [], start
        while k < 0xFFFFFFFA:
            out.append(k)
            k = table[k]
        return out

    dirs = b"".join(sector(k) for k in chain(dir0, fat))
    entries = []
    for off in range(0, len(dirs), 128):
        e = dirs[off:off + 128]
        nlen = struct.unpack_from("<H", e, 0x40)[0]
        name = e[:max(0, nlen - 2)].decode("utf-16-le")
        etype = e[0x42]
        start, size = struct.unpack_from("<II", e, 0x74)
        entries.append((name, etype, start, size))
    root = entries[0]
    for name, etype, start, size in entries:
        if etype != 2 or name not in want:
            continue
        if size >= cutoff:
            return b"".join(sector(k) for k in chain(start, fat))[:size]
        mini = b"".join(sector(k) for k in chain(root[2], fat))
        mfat = []
        for k in chain(mfat0, fat):
            mfat += struct.unpack(f"<{per}I", sector(k))
        return b"".join(mini[k * msz:(k + 1) * msz] for k in chain(start, mfat))[:size]
    raise ValueError("no Workbook stream")


# --------------------------------------------------------------------------
# BIFF8
# --------------------------------------------------------------------------
def _records(wb: bytes):
    off = 0
    while off + 4 <= len(wb):
        rtype, rlen = struct.unpack_from("<HH", wb, off)
        yield rtype, wb[off + 4:off + 4 + rlen]
        off += 4 + rlen


def _rk_value(rk: int) -> float:
    if rk & 2:
        v = float(struct.unpack("<i", struct.pack("<I", rk & 0xFFFFFFFC))[0] >> 2)
    else:
        v = struct.unpack("<d", struct.pack("<Q", (rk & 0xFFFFFFFC) << 32))[0]
    return v / 100.0 if rk & 1 else v


def _shared_strings(parts):
    """SST payload split over the SST record and its CONTINUE records."""
    head = parts[0]
    n_unique = struct.unpack_from("<I", head, 4)[0]
    parts = [head[8:]] + list(parts[1:])
    p, off = 0, 0
    out = []

    def take(n):
        nonlocal p, off
        buf = b""
        while len(buf) < n:
            if off >= len(parts[p]):
                p, off = p + 1, 0
            k = min(n - len(buf), len(parts[p]) - off)
            buf += parts[p][off:off + k]
            off += k
        return buf

    for _ in range(n_unique):
        if off >= len(parts[p]):
            p, off = p + 1, 0
        cch = struct.unpack("<H", take(2))[0]
        flags = take(1)[0]
        runs = struct.unpack("<H", take(2))[0] if flags & 0x08 else 0
        ext = struct.unpack("<I", take(4))[0] if flags & 0x04 else 0
        chars, wide = [], flags & 0x01
        left = cch
        while left:
            if off >= len(parts[p]):       # the characters continue in the next record,
                p, off = p + 1, 0          # which restates the high-byte flag
                wide = parts[p][0] & 0x01
                off = 1
            room = len(parts[p]) - off
            n = min(left, room // 2 if wide else room)
            raw = parts[p][off:off + (2 * n if wide else n)]
            off += len(raw)
            chars.append(raw.decode("utf-16-le") if wide else raw.decode("latin-1"))
            left -= n
        take(4 * runs)
        take(ext)
        out.append("".join(chars))
    return out


def sheet_cells(path: str):
    """{(row, col): str | float} of the first worksheet."""
    wb = _stream(open(path, "rb").read())
    sst, sst_parts, cells = [], None, {}
    depth, sheet = 0, 0
    last = None
    for rtype, data in _records(wb):
        if rtype == 0x0809:                      # BOF
            depth += 1
            if struct.unpack_from("<H", data, 2)[0] == 0x0010:
                sheet += 1
        elif rtype == 0x000A:                    # EOF
            depth -= 1
            if sheet == 1 and depth == 0:
                break
        if rtype == 0x00FC:
            sst_parts = [data]
        elif rtype == 0x003C and last == "sst":
            sst_parts.append(data)
            continue
        elif sst_parts is not None and not sst:
            sst = _shared_strings(sst_parts)
        last = "sst" if rtype == 0x00FC else None
        if sheet != 1:
            continue
        if rtype == 0x00FD:
            r, c, _, i = struct.unpack_from("<HHHI", data)
            cells[(r, c)] = sst[i]
        elif rtype == 0x0203:
            r, c, _, v = struct.unpack_from("<HHHd", data)
            cells[(r, c)] = v
        elif rtype == 0x027E:
            r, c, _, rk = struct.unpack_from("<HHHI", data)
            cells[(r, c)] = _rk_value(rk)
        elif rtype == 0x00BD:
            r, c0 = struct.unpack_from("<HH", data)
            c1 = struct.unpack_from("<H", data, len(data) - 2)[0]
            for k in range(c1 - c0 + 1):
                _, rk = struct.unpack_from("<HI", data, 4 + 6 * k)
                cells[(r, c0 + k)] = _rk_value(rk)
    return cells


def read_fixations(path: str):
    """read_xls_fixations.m:84-138 on the walker's cells: (data, names, trials),
    data[s][t] an array of [x y] (or [x y d]) rows."""
    cells = sheet_cells(path)
    r0 = min(r for r, _ in cells)
    c0 = min(c for _, c in cells)
    nrow = max(r for r, _ in cells) - r0 + 1
    ncol = max(c for _, c in cells) - c0 + 1
    head = [cells.get((r0, c0 + c)) for c in range(ncol)]
    col = {h: head.index(h) + c0 for h in ("SubjectID", "TrialID", "FixX", "FixY") if h in head}
    if len(col) != 4 or any(head.count(h) != 1 for h in col):
        raise ValueError("header cells")
    fd = head.index("FixD") + c0 if head.count("FixD") == 1 else None

    def ident(v):
        return v if isinstance(v, str) else "%g" % v

    names, trials, data = [], [], []
    for r in range(r0 + 1, r0 + nrow):
        row = [cells.get((r, col["FixX"])), cells.get((r, col["FixY"]))]
        if fd is not None:
            row.append(cells.get((r, fd)))
        if any(isinstance(v, str) for v in row):
            raise ValueError("a fixation value is text")
        sid, tid = ident(cells.get((r, col["SubjectID"]))), ident(cells.get((r, col["TrialID"])))
        if sid not in names:
            names.append(sid)
            trials.append([])
            data.append([])
        s = names.index(sid)
        if tid not in trials[s]:
            trials[s].append(tid)
            data[s].append([])
        data[s][trials[s].index(tid)].append(row)
    return [[np.array(t, dtype=float) for t in subj] for subj in data], names, trials
