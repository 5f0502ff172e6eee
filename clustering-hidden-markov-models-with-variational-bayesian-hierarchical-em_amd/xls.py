"""Fixation data from Excel 97-2003 workbooks (the C1 demo's
input, demo/vbdemo_face.m:9).

:func:`read_xls_fixations` restates src/util/read_xls_fixations.m:47-138 (header
cells SubjectID, TrialID, FixX, FixY, optional FixD; data grouped by subject and
trial in order of appearance).  MATLAB's ``xlsread`` is replaced by a small
reader of the BIFF8 format inside an OLE2 compound file (no xlrd here): the
first worksheet's NUMBER, RK, MULRK, LABELSST and LABEL cells, strings from the
shared string table (SST + CONTINUE records).  Host-side input plumbing; the
sequences feed :func:`vbhem_amd.vbhmm.vbhmm_fb`.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Tuple

import numpy as np

_FREE, _ENDCHAIN = 0xFFFFFFFF, 0xFFFFFFFE


def _cfb_stream(data: bytes, names=("Workbook", "Book")) -> bytes:
    """The named stream of an OLE2 compound file (MS-CFB): header, FAT from the
    DIFAT, directory chain, mini stream for small streams."""
    if data[:8] != bytes.fromhex("d0cf11e0a1b11ae1"):
        raise ValueError("not an OLE2 compound file (.xls of Excel 97-2003)")
    ssz = 1 << struct.unpack_from("<H", data, 0x1E)[0]
    msz = 1 << struct.unpack_from("<H", data, 0x20)[0]
    ndir_first = struct.unpack_from("<I", data, 0x30)[0]
    cutoff = struct.unpack_from("<I", data, 0x38)[0]
    mfat_first, nmfat = struct.unpack_from("<II", data, 0x3C)
    difat_first, ndifat = struct.unpack_from("<II", data, 0x44)
    difat = list(struct.unpack_from("<109I", data, 0x4C))
    sec = lambda i: data[(i + 1) * ssz:(i + 2) * ssz]
    d, n = difat_first, ndifat
    while n > 0 and d not in (_FREE, _ENDCHAIN):
        ids = struct.unpack_from(f"<{ssz // 4}I", sec(d))
        difat.extend(ids[:-1])
        d, n = ids[-1], n - 1
    fat = []
    for i in difat:
        if i in (_FREE, _ENDCHAIN):
            continue
        fat.extend(struct.unpack_from(f"<{ssz // 4}I", sec(i)))

    def chain(start, table, size, get):
        out, s, guard = [], start, 0
        while s not in (_FREE, _ENDCHAIN) and s < len(table) and guard <= len(table):
            out.append(get(s))
            s, guard = table[s], guard + 1
        return b"".join(out)[:size] if size is not None else b"".join(out)

    dirs = chain(ndir_first, fat, None, sec)
    entries = []
    for o in range(0, len(dirs) - 127, 128):
        nlen = struct.unpack_from("<H", dirs, o + 0x40)[0]
        name = dirs[o:o + max(0, nlen - 2)].decode("utf-16-le", "replace")
        typ = dirs[o + 0x42]
        start, size = struct.unpack_from("<II", dirs, o + 0x74)
        entries.append((name, typ, start, size))
    root = next(e for e in entries if e[1] == 5)
    for name, typ, start, size in entries:
        if typ == 2 and name in names:
            if size >= cutoff:
                return chain(start, fat, size, sec)
            mini = chain(root[2], fat, root[3], sec)
            mfat = list(struct.unpack_from(f"<{(nmfat * ssz) // 4}I",
                                           chain(mfat_first, fat, nmfat * ssz, sec)))
            return chain(start, mfat, size, lambda i: mini[i * msz:(i + 1) * msz])
    raise ValueError("no Workbook stream in the compound file")


def _rk(v: int) -> float:
    """RK number: 30-bit integer or the top 30 bits of an IEEE double, /100 if flagged."""
    if v & 2:
        x = float(v >> 2 if v < 0x80000000 else (v >> 2) - (1 << 30))
    else:
        x = struct.unpack("<d", struct.pack("<Q", (v & 0xFFFFFFFC) << 32))[0]
    return x / 100.0 if v & 1 else x


def _read_sst(parts: List[bytes]) -> List[str]:
    """Shared strings: SST record + CONTINUE parts; a string's characters may run
    into the next part, which then restarts with an option byte."""
    out: List[str] = []
    p, k = 0, 0
    buf = parts[0]
    _, nuniq = struct.unpack_from("<II", buf, 0)
    p = 8

    def need(n):
        nonlocal buf, p, k
        if p + n > len(buf) and k + 1 < len(parts):
            buf, p, k = parts[k + 1], 0, k + 1

    for _ in range(nuniq):
        need(3)
        nch, flags = struct.unpack_from("<HB", buf, p)
        p += 3
        rich = ext = 0
        if flags & 8:
            rich = struct.unpack_from("<H", buf, p)[0]
            p += 2
        if flags & 4:
            ext = struct.unpack_from("<I", buf, p)[0]
            p += 4
        wide = flags & 1
        chars = []
        left = nch
        while left > 0:
            if p >= len(buf):
                k += 1
                buf, p = parts[k], 0
                wide = buf[p] & 1
                p += 1
            w = 2 if wide else 1
            take = min(left, (len(buf) - p) // w)
            raw = buf[p:p + take * w]
            chars.append(raw.decode("utf-16-le" if wide else "latin-1"))
            p += take * w
            left -= take
        out.append("".join(chars))
        skip = 4 * rich + ext
        while skip > 0:
            if p >= len(buf):
                k += 1
                buf, p = parts[k], 0
            s = min(skip, len(buf) - p)
            p += s
            skip -= s
    return out


def read_xls_cells(path: str) -> Dict[Tuple[int, int], object]:
    """{(row, col): value} of the first worksheet (0-based), values float or str."""
    wb = _cfb_stream(open(path, "rb").read())
    recs = []
    o = 0
    while o + 4 <= len(wb):
        typ, ln = struct.unpack_from("<HH", wb, o)
        recs.append((typ, wb[o + 4:o + 4 + ln]))
        o += 4 + ln
    sst: List[str] = []
    cells: Dict[Tuple[int, int], object] = {}
    bof_depth, sheet = 0, -1
    i = 0
    while i < len(recs):
        typ, d = recs[i]
        if typ == 0x0809:                                   # BOF
            bof_depth += 1
            if struct.unpack_from("<H", d, 2)[0] == 0x0010:   # worksheet substream
                sheet += 1
        elif typ == 0x000A:                                 # EOF
            bof_depth -= 1
            if sheet == 0 and bof_depth == 0:
                break
        elif typ == 0x00FC:                                 # SST (+ CONTINUE)
            parts = [d]
            while i + 1 < len(recs) and recs[i + 1][0] == 0x003C:
                i += 1
                parts.append(recs[i][1])
            sst = _read_sst(parts)
        elif sheet == 0:
            if typ == 0x0203:                               # NUMBER
                r, c = struct.unpack_from("<HH", d, 0)
                cells[(r, c)] = struct.unpack_from("<d", d, 6)[0]
            elif typ == 0x027E:                             # RK
                r, c = struct.unpack_from("<HH", d, 0)
                cells[(r, c)] = _rk(struct.unpack_from("<I", d, 6)[0])
            elif typ == 0x00BD:                             # MULRK
                r, c0 = struct.unpack_from("<HH", d, 0)
                n = (len(d) - 6) // 6
                for q in range(n):
                    cells[(r, c0 + q)] = _rk(struct.unpack_from("<I", d, 4 + 6 * q + 2)[0])
            elif typ == 0x00FD:                             # LABELSST
                r, c, _, idx = struct.unpack_from("<HHHI", d, 0)
                cells[(r, c)] = sst[idx]
            elif typ == 0x0204:                             # LABEL (BIFF8 string)
                r, c, _, nch = struct.unpack_from("<HHHH", d, 0)
                wide = d[8] & 1
                raw = d[9:9 + nch * (2 if wide else 1)]
                cells[(r, c)] = raw.decode("utf-16-le" if wide else "latin-1")
        i += 1
    return cells


def _name(v) -> str:
    """MATLAB sprintf('%g', x) for numeric IDs (read_xls_fixations.m:110-116)."""
    return v if isinstance(v, str) else "%g" % v


def read_xls_fixations(path: str):
    """(data, subject_names, trial_names) as read_xls_fixations.m: data[s][t] is a
    [T x 2] (or [T x 3] with FixD) float array of the t-th trial of subject s."""
    cells = read_xls_cells(path)
    ncol = 1 + max(c for (r, c) in cells if r == 0)
    headers = [cells.get((0, c)) for c in range(ncol)]

    def col(h, required=True):
        idx = [c for c, x in enumerate(headers) if x == h]
        if len(idx) != 1 and (required or len(idx) > 1):
            raise ValueError(f"error with {h}")
        return idx[0] if idx else None

    SID, TID, FX, FY = col("SubjectID"), col("TrialID"), col("FixX"), col("FixY")
    FD = col("FixD", required=False)
    nrow = 1 + max(r for (r, c) in cells)
    names: List[str] = []
    trials: List[List[str]] = []
    data: List[List[list]] = []
    for r in range(1, nrow):
        if (r, SID) not in cells:
            continue
        cols = [FX, FY] + ([FD] if FD is not None else [])
        vals = [cells.get((r, c)) for c in cols]
        if any(isinstance(v, str) for v in vals):
            raise ValueError("fixation values must be numbers, not text")
        sid, tid = _name(cells[(r, SID)]), _name(cells[(r, TID)])
        if sid not in names:
            names.append(sid)
            trials.append([])
            data.append([])
        s = names.index(sid)
        if tid not in trials[s]:
            trials[s].append(tid)
            data[s].append([])
        data[s][trials[s].index(tid)].append([float(v) for v in vals])
    data_np = [[np.asarray(t, dtype=np.float64) for t in subj] for subj in data]
    return data_np, names, trials
