"""Copies the Pinot-WRITTEN index bytes the reference keeps as test data into tests/golden/pinot_written/.

Run in the build container (the reference is not on the GPU box); the outputs are committed data files:
  padding{Null,Old,Percent}/   v1 segment directories (metadata.properties, <col>.dict, <col>.sv.unsorted.fwd),
                               unpacked from pinot-core/src/test/resources/data/padding*.tar.gz (tarfile, data only)
  fixedByte{Raw,Compressed}.v2, fixedByteSVRDoubles.v1
                               DOUBLE fixed-byte chunk forward indexes; FixedByteChunkSVForwardIndexTest.java:331-345
                               reads value i as i + 100.2356 (v2, 2000 docs) and i + 0 (v1, 10009 docs)
  varByteStrings{Raw,Compressed}.v2, varByteStrings.v1
                               raw STRING var-byte chunk forward indexes; VarByteChunkSVForwardIndexTest.java:146-161
                               reads doc i as data[i % 4] of {"abcdefghijk", "12456887", "pqrstuv", "500"} (v2, 1000
                               docs, PASS_THROUGH / SNAPPY) and of {"abcde", "fgh", "ijklmn", "12345"} (v1; its
                               5 chunks of 1009 rows hold 5003 docs, the last chunk 967)
"""
import os
import shutil
import tarfile

SRC = "/root/reference/pinot-core/src/test/resources/data"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pinot_written")


def main():
    os.makedirs(DST, exist_ok=True)
    for name in ("paddingNull", "paddingOld", "paddingPercent"):
        with tarfile.open(os.path.join(SRC, name + ".tar.gz")) as t:
            for m in t.getmembers():
                if m.isfile() and not m.name.endswith("creation.meta"):
                    data = t.extractfile(m).read()
                    out = os.path.join(DST, m.name)
                    os.makedirs(os.path.dirname(out), exist_ok=True)
                    with open(out, "wb") as f:
                        f.write(data)
    for name in ("fixedByteRaw.v2", "fixedByteCompressed.v2", "fixedByteSVRDoubles.v1", "varByteStringsRaw.v2",
                 "varByteStringsCompressed.v2", "varByteStrings.v1"):
        shutil.copyfile(os.path.join(SRC, name), os.path.join(DST, name))


if __name__ == "__main__":
    main()
