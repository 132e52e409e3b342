"""Fixture generator (test infrastructure): the inputs of the reference's
real-data run, Heavy_metals/processed_data.RDS (run_script.R:8-12), as a
compressed npz under tests/golden/.

The RDS is R's serialization format (gzip'd XDR, version 3).  It is read by
the minimal parser below, which only decodes data (vectors, lists, pairlist
attributes, symbols, strings) and executes nothing from the file; any other
item type raises.  Run from the repo root:  python tests/golden/make_heavy_metals.py
"""
import gzip
import struct
import sys
from pathlib import Path

import numpy as np

SRC = Path("/root/reference/Heavy_metals/processed_data.RDS")
OUT = Path(__file__).resolve().parent / "heavy_metals.npz"

NILVALUE, REFSXP, NILSXP, SYMSXP, LISTSXP = 254, 255, 0, 1, 2
LGLSXP, INTSXP, REALSXP, STRSXP, VECSXP, CHARSXP = 10, 13, 14, 16, 19, 9
NA_INT = -(2 ** 31)
ALTREP = 238


class Reader:
    def __init__(self, buf):
        self.b, self.p, self.refs = buf, 0, []

    def i32(self):
        v = struct.unpack_from(">i", self.b, self.p)[0]
        self.p += 4
        return v

    def length(self):
        n = self.i32()
        if n == -1:
            hi, lo = self.i32(), self.i32()
            n = (hi << 32) + lo
        return n

    def header(self):
        assert self.b[:2] == b"X\n", "not an XDR RDS"
        self.p = 2
        version = self.i32()
        self.i32()  # writer R version
        self.i32()  # minimal reader version
        if version == 3:
            nelen = self.i32()
            self.p += nelen  # native encoding
        return version

    def item(self):
        return self.item_from(self.i32())

    def item_from(self, flags):
        t = flags & 0xFF
        has_attr, has_tag = bool(flags & (1 << 9)), bool(flags & (1 << 10))
        if t == NILVALUE:
            return None
        if t == REFSXP:
            return self.refs[(flags >> 8) - 1]
        if t == ALTREP:  # info (class, package, type), state, attributes
            info = self.item()
            state = self.item()
            attrs = self.item()
            cls = info[0][1] if isinstance(info, dict) and isinstance(info.get(0), tuple) else None
            if cls in ("compact_intseq", "compact_realseq"):
                n, start, step = state["value"][:3]
                v = start + step * np.arange(int(n))
                v = v.astype(np.int64) if cls == "compact_intseq" else v.astype(np.float64)
                return {"type": INTSXP if cls == "compact_intseq" else REALSXP, "value": v,
                        "attrs": attrs or {}}
            if cls is not None and cls.startswith("wrap_"):
                inner = state[0]
                if attrs:
                    inner = dict(inner, attrs=attrs)
                return inner
            if cls == "deferred_string":  # as.character() of a numeric vector, done lazily in R
                src = state[0]["value"]
                v = [str(int(x)) if float(x).is_integer() else repr(float(x)) for x in src]
                return {"type": STRSXP, "value": v, "attrs": attrs or {}}
            raise ValueError(f"ALTREP class {cls} not supported by this data-only reader")
        if t == SYMSXP:
            name = self.item()
            self.refs.append(("sym", name))
            return ("sym", name)
        if t == CHARSXP:
            n = self.i32()
            if n == -1:
                return None
            s = self.b[self.p:self.p + n].decode("utf-8", "replace")
            self.p += n
            return s
        if t == LISTSXP:  # pairlist (attributes): tag -> value
            out = {}
            while True:
                attr = self.item() if has_attr else None
                tag = self.item() if has_tag else None
                val = self.item()
                out[tag[1] if tag else len(out)] = val
                nxt = self.i32()
                if (nxt & 0xFF) == NILVALUE:
                    break
                if (nxt & 0xFF) != LISTSXP:  # dotted pair: the CDR is an ordinary item
                    out["cdr"] = self.item_from(nxt)
                    break
                has_attr, has_tag = bool(nxt & (1 << 9)), bool(nxt & (1 << 10))
            return out
        if t in (INTSXP, LGLSXP):
            n = self.length()
            v = np.frombuffer(self.b, ">i4", n, self.p).astype(np.int64)
            self.p += 4 * n
        elif t == REALSXP:
            n = self.length()
            v = np.frombuffer(self.b, ">f8", n, self.p).astype(np.float64)
            self.p += 8 * n
        elif t == STRSXP:
            n = self.length()
            v = [self.item() for _ in range(n)]
        elif t == VECSXP:
            n = self.length()
            v = [self.item() for _ in range(n)]
        else:
            raise ValueError(f"RDS item type {t} not supported by this data-only reader")
        attrs = self.item() if has_attr else {}
        return {"type": t, "value": v, "attrs": attrs or {}}


def main():
    r = Reader(gzip.decompress(SRC.read_bytes()))
    assert r.header() == 3
    top = r.item()
    names = top["attrs"]["names"]["value"]
    obj = dict(zip(names, top["value"]))
    locs = obj["observed_locs"]
    dim = locs["attrs"]["dim"]["value"]
    observed_locs = locs["value"].reshape(int(dim[1]), int(dim[0])).T  # R column-major
    observed_field = obj["observed_field"]["value"]
    xl = obj["X_locs"]
    cols = xl["attrs"]["names"]["value"]
    num_names, num, fac_names, fac_codes, fac_levels = [], [], [], [], []
    for nm, col in zip(cols, xl["value"]):
        cls = col["attrs"].get("class", {}).get("value", [])
        if "factor" in cls:
            fac_names.append(nm)
            fac_codes.append(col["value"].astype(np.int32))  # 1-based level codes
            fac_levels.append(np.array(col["attrs"]["levels"]["value"]))
        else:
            num_names.append(nm)
            num.append(col["value"])
    payload = {
        "observed_locs": observed_locs, "observed_field": observed_field,
        "X_num": np.column_stack(num), "X_num_names": np.array(num_names),
        "X_fac_names": np.array(fac_names), "column_order": np.array(cols),
    }
    for nm, c, lv in zip(fac_names, fac_codes, fac_levels):
        payload[f"fac_{nm}"] = c
        payload[f"levels_{nm}"] = lv
    for k in ("X_locs_mean", "X_locs_sd"):
        if k in obj:
            payload[k] = obj[k]["value"]
    np.savez_compressed(OUT, **payload)
    print(f"wrote {OUT} ({OUT.stat().st_size / 1e6:.1f} MB): locs {observed_locs.shape}, "
          f"{len(num_names)} numeric + {len(fac_names)} factor covariates "
          f"({[len(l) for l in fac_levels]} levels)", file=sys.stderr)


if __name__ == "__main__":
    main()
