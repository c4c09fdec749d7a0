"""Extract the reference CityHash KAT (cityhash/test/city.cc) as a data fixture.

The reference test hashes data[offset : offset+len] for len=i, offset=i*i,
i in [0, 298], plus (offset 0, len 1 MiB), where `data` is the deterministic
buffer built by setup() (cityhash/test/city.cc:46-58; restated in
tests/kat_data.py).  Expected outputs live in testdata[300][16]
(cityhash/test/city.cc:63-1265): column 0 = CityHash64, column 1 =
CityHash64WithSeed(kSeed0), column 2 = CityHash64WithSeeds(kSeed0, kSeed1).

Only the numbers are written (tests/golden/cityhash64_kat.json).  Run once in
the build container; /root/reference is not needed afterwards.
"""
import json
import re
import sys

SRC = "/root/reference/cityhash/test/city.cc"


def main(out="tests/golden/cityhash64_kat.json"):
    text = open(SRC).read()
    body = text[text.index("testdata[kTestSize][16]"):text.index("void Check(")]
    rows = re.findall(r"\{([^{}]*)\}", body)
    cases = []
    for i, row in enumerate(rows):
        vals = [int(v, 16) for v in re.findall(r"C\(([0-9a-f]+)\)", row)]
        assert len(vals) == 16, (i, len(vals))
        offset, length = (i * i, i) if i < len(rows) - 1 else (0, 1 << 20)
        cases.append({"offset": offset, "len": length,
                      "cityhash64": "%016x" % vals[0],
                      "cityhash64_seed": "%016x" % vals[1],
                      "cityhash64_seeds": "%016x" % vals[2]})
    assert len(cases) == 300
    json.dump({"source": "cityhash/test/city.cc:63-1265 (column 0,1,2), "
                         "inputs from setup() :46-58 with a=9, b=777, 1 MiB",
               "cases": cases}, open(out, "w"), indent=0)
    print("wrote", out, len(cases))


if __name__ == "__main__":
    main(*sys.argv[1:])
