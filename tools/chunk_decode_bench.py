"""Pin-time decode of compressed raw chunks (SNAPPY / LZ4 / LZ4_LENGTH_PREFIXED) on one MI355X.

Builds one SSB-sized segment (6M rows) per (codec, data shape) with a raw LONG column in 1000-doc chunks
(ForwardIndexConfig default), loads it `--reps` times through phip_segment_load, and prints one JSON line
per case: compressed / decoded bytes and the wall time of the load (H2D of the compressed blob included).
Kernel-only time comes from `rocprofv3 --kernel-trace --stats` over this script (chunk_decode_kernel).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pinot_amd import _lib  # noqa: E402
from pinot_amd.engine.segment import GpuSegment  # noqa: E402
from pinot_amd.segment.creator import SegmentCreator  # noqa: E402
from pinot_amd.spi import DataType  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=6_000_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    lib = _lib.load()
    _lib.check(lib.phip_init(None, 0))
    rng = np.random.default_rng(7)
    n = args.rows
    shapes = {
        "revenue_like": rng.integers(100_000, 10_000_000, n),        # SSB lo_revenue range, ~3 incompressible bytes
        "lowcard": rng.integers(0, 50, n) * 100,                      # lo_quantity-like: compresses well
    }
    for shape, vals in shapes.items():
        for codec in ("LZ4", "LZ4_LENGTH_PREFIXED", "SNAPPY"):
            c = SegmentCreator(f"{shape}_{codec}", no_dictionary_columns=["M"], raw_compression={"M": codec})
            c.add_column("M", DataType.LONG, vals)
            seg = c.build()
            comp = len(seg.columns["M"].forward)
            times = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                g = GpuSegment(seg)
                times.append(time.perf_counter() - t0)
                g.destroy()
            med = float(np.median(times))
            print(json.dumps({"shape": shape, "codec": codec, "rows": n, "compressed_bytes": comp,
                              "decoded_bytes": 8 * n, "ratio": round(8 * n / comp, 3),
                              "load_ms_p50": round(med * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
