"""Round 6 diagnostic for the round-5 peer-region failure: what becomes of
device memory allocated uncached / fine-grained and then freed, and do fp64 atomics sum exactly on it?

Prints one JSON object.  Scenarios:
  direct   - hipMalloc / uncached / fine-grained blocks of several sizes: allocation range, flags, fp64 + u32
             atomic sums (wrong-slot counts);
  reuse    - for each special kind and region size: allocate, free, then 24 hipMalloc blocks of the sizes the
             engine's block cache uses; which land inside the freed range, their allocation base / flags, and
             their atomic sums;
  coreside - a special block kept alive while small hipMalloc blocks are taken: do they share its allocation?
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests", "native"))


def main():
    import build_probe
    lib = ctypes.CDLL(build_probe.build())
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.ucp_alloc.argtypes = [ctypes.c_int, sz, ctypes.POINTER(vp)]
    lib.ucp_free.argtypes = [vp]
    lib.ucp_range.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(sz)]
    lib.ucp_flags.argtypes = [vp, ctypes.POINTER(ctypes.c_uint)]
    lib.ucp_atomics.argtypes = [vp, ctypes.c_longlong, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong)]
    KIND = {0: "hipMalloc", 1: "uncached", 2: "finegrained"}

    def alloc(kind, nbytes):
        p = vp()
        rc = lib.ucp_alloc(kind, nbytes, ctypes.byref(p))
        assert rc == 0, (kind, nbytes, rc)
        return p.value

    def info(p, nbytes):
        b, s, f = vp(), sz(), ctypes.c_uint()
        rc1 = lib.ucp_range(p, ctypes.byref(b), ctypes.byref(s))
        rc2 = lib.ucp_flags(p, ctypes.byref(f))
        nslots = max(1, min(nbytes // 8, 4096))
        wf, wu = ctypes.c_longlong(), ctypes.c_longlong()
        rc3 = lib.ucp_atomics(p, nslots, ctypes.byref(wf), ctypes.byref(wu))
        return {"ptr": hex(p), "base": hex(b.value or 0), "range": s.value, "flags": f.value, "rc": [rc1, rc2, rc3],
                "slots": nslots, "wrong_f64": wf.value, "wrong_u32": wu.value}

    out = {"direct": [], "reuse": [], "coreside": []}
    for kind in (0, 1, 2):
        for nbytes in (64 << 10, 1 << 20, 2359296, 8 << 20):
            p = alloc(kind, nbytes)
            out["direct"].append({"kind": KIND[kind], "bytes": nbytes, **info(p, nbytes)})
            lib.ucp_free(p)
    sizes = [256, 4096, 65536, 1 << 20, 2 << 20, 4 << 20]
    for kind in (1, 2):
        for nbytes in (64 << 10, 1 << 20, 2359296, 8 << 20):
            r = alloc(kind, nbytes)
            lib.ucp_free(r)
            blocks, rows = [], []
            for i in range(24):
                b = sizes[i % len(sizes)]
                p = alloc(0, b)
                blocks.append(p)
                inside = r <= p < r + nbytes
                row = {"bytes": b, "inside_freed": inside, **info(p, b)}
                rows.append(row)
            for p in blocks:
                lib.ucp_free(p)
            out["reuse"].append({"kind": KIND[kind], "region_bytes": nbytes, "region": hex(r),
                                 "n_inside": sum(x["inside_freed"] for x in rows),
                                 "n_wrong_f64": sum(x["wrong_f64"] > 0 for x in rows),
                                 "n_wrong_u32": sum(x["wrong_u32"] > 0 for x in rows),
                                 "blocks": rows})
    for kind in (1, 2):
        r = alloc(kind, 64 << 10)
        rb, rs = vp(), sz()
        lib.ucp_range(r, ctypes.byref(rb), ctypes.byref(rs))
        rows = []
        blocks = []
        for b in (256, 4096, 65536, 65536):
            p = alloc(0, b)
            blocks.append(p)
            row = {"bytes": b, **info(p, b)}
            row["shares_special_allocation"] = int(row["base"], 16) == (rb.value or 0)
            rows.append(row)
        for p in blocks:
            lib.ucp_free(p)
        lib.ucp_free(r)
        out["coreside"].append({"kind": KIND[kind], "special": hex(r), "special_base": hex(rb.value or 0),
                                "special_range": rs.value, "blocks": rows})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
