"""Round 6: does memory that lived as ordinary (cached) device memory and is then allocated uncached /
fine-grained show its OLD contents to the GPU's loads?  (tests/native/uc_probe.hip, ucp_stale.)  One JSON
object: per (kind, size, flush): elements != the new pattern for system-scope loads / ordinary loads /
hipMemcpy, elements equal to the old pattern, and whether the special block got the freed VA."""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests", "native"))


def main():
    import build_probe
    lib = ctypes.CDLL(build_probe.build())
    lib.ucp_stale.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_longlong)]
    rows = []
    for kind in (1, 2):
        for nbytes in (65536, 2359296, 2 << 20, 4 << 20, 4718592, 8 << 20):
            for flush in (0, 4, 0, 4, 1, 2, 3):
                c = (ctypes.c_longlong * 7)()
                rc = lib.ucp_stale(kind, nbytes, flush, c)
                rows.append({"kind": ["", "uncached", "finegrained"][kind], "bytes": nbytes, "flush": flush, "rc": rc,
                             "bad_sys": c[0], "bad_plain": c[1], "bad_memcpy": c[2],
                             "old_sys": c[3], "old_plain": c[4], "old_memcpy": c[5], "same_va": c[6]})
                print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
