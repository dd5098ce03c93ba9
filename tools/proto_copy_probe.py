"""What the wire format does with a payload ("D2H straight
into the returned bytes").  Measures, on the host, for a payload of the
ResNet-50 planes size and 100 MB:
  * whether NamedTensor.data_bytes accepts anything but `bytes`
    (bytearray / memoryview / ndarray) -- it does not;
  * the cost of assigning a `bytes` to data_bytes (protobuf copies it into its
    own arena) and of SerializeToString (a second copy), against
  * one pinned-staging -> bytes copy (what forward_batch does after the D2H).
Prints one JSON line.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from openfl_amd import protocols as P  # noqa: E402


def best(fn, reps=5):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return min(t)


def main():
    out = {"accepts": {}}
    nt = P.NamedTensor()
    for v in (bytearray(b"ab"), memoryview(b"ab"), np.frombuffer(b"ab", np.uint8)):
        try:
            nt.data_bytes = v
            out["accepts"][type(v).__name__] = True
        except TypeError:
            out["accepts"][type(v).__name__] = False
    for n in (25_610_152, 100_000_000):  # ResNet-50 8-bit planes; 100 MB
        staging = np.random.default_rng(0).integers(0, 255, n, dtype=np.uint8)
        b = staging.tobytes()
        t_copy = best(lambda: staging.tobytes())
        t_assign = best(lambda: setattr(nt, "data_bytes", b))
        nt.data_bytes = b
        t_ser = best(lambda: nt.SerializeToString())
        out[str(n)] = {"staging_to_bytes_ms": round(1e3 * t_copy, 2), "assign_data_bytes_ms": round(1e3 * t_assign, 2),
                       "serialize_ms": round(1e3 * t_ser, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
