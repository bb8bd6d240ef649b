"""Property-column helpers for the MVT cross-check of the property decode (SURVEY.md §8(f) row 3;
the property half of CovtParserTest.compareTiles, CovtParserTest.java:62-90).

* ``mvt_properties``: feature tags of a Mapbox Vector Tile (spec v2: layer keys, values, feature
  tag pairs) as ``{layer_name: [{key: value}, ...]}`` -- used only by ``tests/golden/make_golden.py``
  on the reference's MVT fixtures (``test/fixtures/omt/mvt``).
* ``values_digest``: order-preserving SHA-256 of a per-feature value list (None = absent), the
  form in which both the MVT properties and the decoded COVT property columns are compared.
* ``candidate_keys``: MVT keys a decoded COVT (sub)column may correspond to: the column name, and
  for a Gen C localized-dictionary language stream ``L`` of column ``name`` the keys ``name``
  (L == "name"), ``name:L`` and ``name_L``.
"""
from __future__ import annotations

import hashlib
import struct

import numpy as np

from covt_geom import _fields, _packed, _zz


def _value(v: bytes):
    out = None
    for f, wt, x in _fields(v):
        if f == 1:
            out = x.decode("utf-8")
        elif f == 2:
            out = float(struct.unpack("<f", struct.pack("<I", x))[0])
        elif f == 3:
            out = float(struct.unpack("<d", struct.pack("<Q", x))[0])
        elif f == 4:
            out = x - (1 << 64) if x >= 1 << 63 else x
        elif f == 5:
            out = x
        elif f == 6:
            out = _zz(x)
        elif f == 7:
            out = bool(x)
    return out


def mvt_properties(data: bytes):
    out = {}
    for f, wt, v in _fields(data):
        if f != 3 or wt != 2:
            continue
        name, keys, vals, feats = None, [], [], []
        for lf, lwt, lv in _fields(v):
            if lf == 1:
                name = lv.decode("utf-8")
            elif lf == 3:
                keys.append(lv.decode("utf-8"))
            elif lf == 4:
                vals.append(_value(lv))
            elif lf == 2:
                tags = []
                for ff, fwt, fv in _fields(lv):
                    if ff == 2:
                        tags = _packed(fv) if fwt == 2 else [fv]
                feats.append(tags)
        out[name] = [{keys[t[i]]: vals[t[i + 1]] for i in range(0, len(t), 2)} for t in feats]
    return out


def _canon(x) -> bytes:
    if x is None:
        return b"N"
    if isinstance(x, bool):
        return b"b1" if x else b"b0"
    if isinstance(x, (int, np.integer)):
        return b"i" + str(int(x)).encode()
    if isinstance(x, (float, np.floating)):
        return b"f" + np.float32(x).tobytes().hex().encode()
    return b"s" + str(x).encode("utf-8")


def values_digest(values) -> str:
    h = hashlib.sha256()
    for x in values:
        c = _canon(x)
        h.update(struct.pack("<I", len(c)))
        h.update(c)
    return h.hexdigest()


def candidate_keys(column: str, lang):
    if lang is None:
        return [column]
    if lang == "name":
        return ["name"]
    return [column + ":" + lang, column + "_" + lang]
