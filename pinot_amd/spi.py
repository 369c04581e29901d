"""Data types and constants shared by the host mirror and the C-ABI.

Mirrors ``FieldSpec.DataType`` (pinot-spi/src/main/java/org/apache/pinot/spi/data/FieldSpec.java)
restricted to the single-value stored types on the hot path, and the numeric codes used by
``include/pinot_hip.h`` (PHIP_TYPE_*).
"""
import enum

import numpy as np


class DataType(enum.IntEnum):
    # values == PHIP_TYPE_* in include/pinot_hip.h
    INT = 0
    LONG = 1
    FLOAT = 2
    DOUBLE = 3
    STRING = 4

    @property
    def numpy_be(self):
        return {DataType.INT: ">i4", DataType.LONG: ">i8", DataType.FLOAT: ">f4",
                DataType.DOUBLE: ">f8"}[self]

    @property
    def numpy(self):
        return {DataType.INT: np.int32, DataType.LONG: np.int64, DataType.FLOAT: np.float32,
                DataType.DOUBLE: np.float64, DataType.STRING: np.str_}[self]

    @property
    def is_numeric(self):
        return self != DataType.STRING

    @property
    def is_integral(self):
        return self in (DataType.INT, DataType.LONG)


class FieldType(enum.Enum):
    DIMENSION = "DIMENSION"
    METRIC = "METRIC"
    DATE_TIME = "DATE_TIME"


# pinot-core/src/main/java/org/apache/pinot/core/plan/DocIdSetPlanNode.java:29
MAX_DOC_PER_CALL = 10_000
# pinot-core/.../plan/maker/InstancePlanMakerImplV2.java:74,78
DEFAULT_MAX_INITIAL_RESULT_HOLDER_CAPACITY = 10_000
DEFAULT_NUM_GROUPS_LIMIT = 100_000
# InstancePlanMakerImplV2 server defaults (pinot-core/.../plan/maker/InstancePlanMakerImplV2.java:80-96) and
# GroupByUtils.MAX_TRIM_THRESHOLD (pinot-core/.../util/GroupByUtils.java:40)
DEFAULT_MIN_SEGMENT_GROUP_TRIM_SIZE = -1
DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE = 5000
DEFAULT_GROUPBY_TRIM_THRESHOLD = 1_000_000
MAX_TRIM_THRESHOLD = 1_000_000_000
# pinot-spi/src/main/java/org/apache/pinot/spi/utils/CommonConstants.java:117
DEFAULT_HYPERLOGLOG_LOG2M = 8


def num_bits_per_value(max_value: int) -> int:
    """``PinotDataBitSet.getNumBitsPerValue`` (pinot-segment-local/.../io/util/PinotDataBitSet.java:61-72)."""
    if max_value <= 1:
        return 1
    return int(max_value).bit_length()
