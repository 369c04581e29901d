"""pinot_amd — MI355X-native single-server segment query hot path for Apache Pinot.

The product is the C-ABI library ``libpinot_hip.so`` (HIP kernels for gfx950 + a C++ host
runtime), declared in ``include/pinot_hip.h``. This Python package is the host-side mirror
of the reference's Java operator surface for that path (plan maker, filter / aggregation /
group-by operators, results blocks) plus the segment writer used to produce test and
benchmark segments in Pinot's on-disk encodings.
"""

__version__ = "0.1.0"
