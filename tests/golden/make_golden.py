#!/usr/bin/env python3
"""Regenerates the committed golden fixtures under tests/golden/ (run in the build container,
where the read-only reference is mounted at /root/reference; the GPU box never runs this).

What it writes (all DATA -- inputs and expected outputs, no reference source):
  tiles/{omt,bing,amazon}/*.covt   the reference's committed COVT fixtures (test/fixtures/*/covt),
                                   byte-identical copies; Gen B variants (omt/3_4_5, amazon_here/*)
                                   are not copied.
  mvt_digests.json                 per OMT tile and layer: SHA-256 of the per-feature geometry and of
                                   the feature ids decoded from the reference's MVT originals
                                   (test/fixtures/omt/mvt/*.mvt) -- independent of any COVT decoder.
                                   Also the oracle-vs-MVT pass list at generation time.
  kats.json                        known-answer vectors from the reference's TS unit tests
                                   (parser/js/test/unit/decoder/decodingUtils.spec.ts), valid subset.
  mvt_prop_digests.json            per OMT tile, layer and MVT key: SHA-256 of the per-feature property
                                   values of the reference's MVT originals (tests/covt_props.py), plus
                                   the oracle's property-column pass list at generation time.
  oracle_streams.json              per tile and Id/Geometry stream: walk record + SHA-256 of the
                                   oracle's decoded bytes (both Id modes) -- regression pin.
  5_16_20.npz                      full decoded arrays of the config-1/2 tile.
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(HERE))

import oracle as O  # noqa: E402
import covt_geom as G  # noqa: E402
import covt_props as P  # noqa: E402

REF = "/root/reference/test/fixtures"
SETS = ("omt", "bing", "amazon")
EXCLUDED_GEN_B = {"omt/3_4_5"}


def copy_tiles():
    for s in SETS:
        dst = os.path.join(HERE, "tiles", s)
        os.makedirs(dst, exist_ok=True)
        for f in sorted(glob.glob(os.path.join(REF, s, "covt", "*.covt"))):
            key = s + "/" + os.path.basename(f)[:-5]
            if key in EXCLUDED_GEN_B:
                continue
            shutil.copyfile(f, os.path.join(dst, os.path.basename(f)))


def layer_names(t: bytes):
    def vu(o):
        r = sh = 0
        while True:
            b = t[o]
            o += 1
            r |= (b & 0x7F) << sh
            sh += 7
            if b < 0x80:
                return r, o

    o = 0
    _, o = vu(o)
    nl, o = vu(o)
    names = []
    for _ in range(nl):
        n, o = vu(o)
        names.append(t[o:o + n].decode())
        o += n
        _, o = vu(o)
        _, o = vu(o)
        nc, o = vu(o)
        tot = 0
        for _ in range(nc):
            n, o = vu(o)
            o += n + 2
            ns, o = vu(o)
            for _ in range(ns):
                n, o = vu(o)
                o += n
                _, o = vu(o)
                bl, o = vu(o)
                o += 1
                tot += bl
        o += tot
    return names


def decode_tile_layers(t: bytes, id_mode=O.ID_FORMAT):
    st, ss = O.walk_tile(t)
    if st:
        return None
    layers = {}
    for s in ss:
        st2, arr, cons = O.decode_stream(t, s, id_mode)
        if st2:
            return None
        layers.setdefault(s.layer, {})[(s.column_kind, s.stream_type)] = (arr, s)
    return layers


def oracle_layer_digests(t: bytes):
    layers = decode_tile_layers(t)
    if layers is None:
        return None
    out = {}
    for L, d in layers.items():
        def g(k):
            return d[(1, k)][0] if (1, k) in d else None

        ice = d[(1, 9)][1].column_type in (3, 4)
        try:
            geom = G.layer_digest(G.assemble(g(4), g(5), g(6), g(7), g(8), g(9), ice))
        except Exception:  # noqa: BLE001 -- inconsistent count streams
            geom = None
        ids = G.ids_digest(d[(0, 1)][0]) if (0, 1) in d else None
        out[L] = (geom, ids)
    return out


def mvt_digests():
    res = {}
    for f in sorted(glob.glob(os.path.join(HERE, "tiles", "omt", "*.covt"))):
        name = os.path.basename(f)[:-5]
        mpath = os.path.join(REF, "omt", "mvt", name + ".mvt")
        if not os.path.exists(mpath):
            continue
        t = open(f, "rb").read()
        mvt = G.mvt_layers(open(mpath, "rb").read())
        ours = oracle_layer_digests(t)
        names = layer_names(t)
        entry = {}
        for L, lname in enumerate(names):
            m = mvt.get(lname)
            if m is None:
                continue
            mg = G.layer_digest([(c, p) for (_, c, p) in m["features"]])
            mi = G.ids_digest([i for (i, _, _) in m["features"]])
            og, oi = (None, None) if ours is None or L not in ours else ours[L]
            entry[str(L)] = {"name": lname, "n_features": len(m["features"]), "geom": mg, "ids": mi,
                             "oracle_geom_match": og == mg, "oracle_ids_match": oi == mi}
        res[name] = entry
    return res


def mvt_prop_digests():
    """{tile: {"mvt": {layer: {key: digest}}, "oracle_pass": [[layer, column name], ...]}} over the
    OMT tiles that have an MVT original; a decoded (sub)column passes when its value digest equals
    the MVT digest of one of its candidate keys."""
    res = {}
    for f in sorted(glob.glob(os.path.join(HERE, "tiles", "omt", "*.covt"))):
        name = os.path.basename(f)[:-5]
        mpath = os.path.join(REF, "omt", "mvt", name + ".mvt")
        if not os.path.exists(mpath):
            continue
        t = open(f, "rb").read()
        mvt = P.mvt_properties(open(mpath, "rb").read())
        dig = {}
        for lname, feats in mvt.items():
            keys = sorted({k for ft in feats for k in ft})
            dig[lname] = {k: P.values_digest([ft.get(k) for ft in feats]) for k in keys}
        names = layer_names(t)
        st, props = O.walk_properties(t)
        passed = []
        for p in props:
            lname = names[p.layer]
            st2, vals = O.property_values(t, p)
            if st2 or lname not in dig:
                continue
            col = O.prop_name(t, p)
            base, lang = (col.split(":", 1) + [None])[:2] if p.lang >= 0 else (col, None)
            d = P.values_digest(vals)
            if any(dig[lname].get(k) == d for k in P.candidate_keys(base, lang)):
                passed.append([p.layer, col])
        res[name] = {"mvt": dig, "oracle_pass": passed, "n_props": len(props)}
    return res


def kats():
    src = "parser/js/test/unit/decoder/decodingUtils.spec.ts"
    return {
        "source": src,
        "varint": [
            {"line": 11, "bytes": [10], "pos": 0, "value": 10, "end": 1},
            {"line": 21, "bytes": [0x80, 0x80, 0x80, 4], "pos": 0, "value": 8388608, "end": 4},
            {"line": 31, "bytes": [0x80, 0x80, 0x80, 0x80, 0x80, 4], "pos": 2, "value": 8388608, "end": 6},
        ],
        "varint_java_divergence": [
            # 7-byte varint (line 42): the TS decoder reads 17592186044416; Java's 4-byte cap
            # (DecodingUtils.java:157-186) stops after 4 bytes -> 0 and pos 6.
            {"line": 42, "bytes": [0x80] * 8 + [4], "pos": 2, "u64_value": 17592186044416, "u64_end": 9,
             "java_value": 0, "java_end": 6},
        ],
        "zigzag_varint": [{"line": 55, "bytes": [155, 4], "pos": 0, "value": -270, "end": 2}],
        "rle": [
            {"line": 68, "bytes": [2, 1, 1, 2, 1, 1], "n": 10, "signed": False,
             "values": [1, 2, 3, 4, 5, 1, 2, 3, 4, 5], "end": 6},
            # run-1 and literal parts of the combined vector (lines 77-103); its run-2 part encodes
            # the delta as zigzag(-1)=1 instead of int8 0xff and is not a valid ORC vector.
            {"line": 85, "bytes": [0x61, 0x00, 0x0E], "n": 100, "signed": True, "values": [7] * 100, "end": 3},
            {"line": 86, "bytes": [0xFB, 4, 6, 12, 14, 22], "n": 5, "signed": True, "values": [2, 3, 6, 7, 11],
             "end": 6},
        ],
    }


def stream_records():
    res = {}
    for s in SETS:
        for f in sorted(glob.glob(os.path.join(HERE, "tiles", s, "*.covt"))):
            t = open(f, "rb").read()
            st, ss = O.walk_tile(t)
            key = s + "/" + os.path.basename(f)[:-5]
            recs = []
            tile_ok = st == 0
            for x in ss:
                row = [x.layer, x.column_kind, x.stream_type, x.encoding, x.column_type, x.num_values,
                       x.byte_length, x.num_bits, x.offset]
                for mode in (O.ID_FORMAT, O.ID_JAVA):
                    st2, arr, cons = O.decode_stream(t, x, mode)
                    tile_ok &= st2 == 0 or mode == O.ID_JAVA
                    row += [st2, cons, hashlib.sha256(arr.tobytes()).hexdigest() if st2 == 0 else None]
                recs.append(row)
            res[key] = {"walk_status": st, "decodable": bool(tile_ok), "size": len(t), "streams": recs}
    return {"columns": ["layer", "column_kind", "stream_type", "encoding", "column_type", "num_values",
                        "byte_length", "num_bits", "offset",
                        "fmt_status", "fmt_consumed", "fmt_sha256", "java_status", "java_consumed",
                        "java_sha256"],
            "tiles": res}


def tile_arrays(name="omt/5_16_20"):
    t = open(os.path.join(HERE, "tiles", name + ".covt"), "rb").read()
    st, ss = O.walk_tile(t)
    assert st == 0
    arrs = {}
    for i, x in enumerate(ss):
        st2, arr, _ = O.decode_stream(t, x, O.ID_FORMAT)
        assert st2 == 0
        arrs["s%03d_L%d_k%d_t%d" % (i, x.layer, x.column_kind, x.stream_type)] = arr
    np.savez_compressed(os.path.join(HERE, "5_16_20.npz"), **arrs)


def main():
    O.build()
    if "--props" in sys.argv:  # regenerate only the property digests
        with open(os.path.join(HERE, "mvt_prop_digests.json"), "w") as f:
            json.dump(mvt_prop_digests(), f, separators=(",", ":"), sort_keys=True)
        return
    copy_tiles()
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(kats(), f, indent=1)
    with open(os.path.join(HERE, "mvt_digests.json"), "w") as f:
        json.dump(mvt_digests(), f, indent=0, sort_keys=True)
    with open(os.path.join(HERE, "oracle_streams.json"), "w") as f:
        json.dump(stream_records(), f, separators=(",", ":"))
    with open(os.path.join(HERE, "mvt_prop_digests.json"), "w") as f:
        json.dump(mvt_prop_digests(), f, separators=(",", ":"), sort_keys=True)
    tile_arrays()
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
