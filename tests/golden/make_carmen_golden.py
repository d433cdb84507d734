"""Generates tests/golden/carmen_ref.json: Carmen log texts and what the
REFERENCE's own CarmenLogReader::Load (C/io/carmen/carmen_reader.cpp, compiled
in place by oracle/ref/Makefile into oracle/_ref/libref_pin.so) returns for
them, as the flat record stream of ref_carmen_load (doubles as hex strings,
bit-exact) plus the sensor ids.  Run in the build container (the reference is
not on the GPU box):  python tests/golden/make_carmen_golden.py
"""
import ctypes as C
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_pin.so")
OUT = os.path.join(ROOT, "tests", "golden", "carmen_ref.json")


def carmen_texts(seed=11):
    """Record types the reader knows (and some it ignores), malformed and
    truncated lines, the sensor-id carry-over of an empty line after ODOM,
    duplicate PARAMs (the first value wins), guessed angle geometry."""
    rng = np.random.default_rng(seed)

    def nums(a):
        return " ".join(repr(float(x)) for x in a)

    lines_a = [
        "PARAM robot_name pioneer",
        "PARAM Laser.MinRange 0.05",
        "PARAM Laser.MaxRange 30.0",
        "PARAM Laser.MaxRange 99.0",
        "PARAM Laser.MinAngle -1.5707963267948966",
        "PARAM Laser.AngleIncrement 0.017453292519943295",
        "PARAM novalue",
        "# comment line",
        "ODOM 1.5 -2.25 0.3 0.1 0.02 0.0 1000.125 nohost 0.5",
        "",
        "ODOM 1.6 -2.2 0.31 0.1 0.02 0.0 1000.25 nohost 0.6",
        "TRUEPOS 1 2 3 4 5 6 7 host 8",
        "RAWLASER1 0 -2.0943951 4.1887902 0.0087266 30.0 0.01 0 5 " + nums(rng.uniform(0.1, 9.0, 5))
        + " 2 0.5 0.7 1001.5 host 1.25",
        "RAWLASER3 0 -1.5707963 3.1415926 0.0174533 20.0 0.01 0 4 1.0 2.0 3.0",  # truncated: zeros follow
        "ROBOTLASER1 0 -1.5707963267948966 3.141592653589793 0.017453292519943295 80.0 0.01 0 181 "
        + nums(rng.uniform(0.05, 15.0, 181)) + " 2.0 -1.0 0.75 1.9 -1.1 0.7 0.2 0.01 0.3 0.4 0.5 1002.0 host 2.0",
        "FLASER 181 " + nums(rng.uniform(0.05, 15.0, 181)) + " 0.5 0.25 -0.3 0.4 0.2 -0.35 1003.0 host 3.0",
        "RLASER 10 " + nums(rng.uniform(0.05, 15.0, 10)) + " 0.5 0.25 -0.3 0.4 0.2 -0.35 1003.5 host 3.5",
        "LASER3 7 " + nums(rng.uniform(0.05, 15.0, 7)),
        "LASER4 3 1 2 3 extra tokens",
        "NMEAGGA 1 2 3",
        "ROBOTLASER2 0 0.0 1.0 0.5 10.0 0.1 0 3 1.5 2.5 3.5 0 0 0 0 0 0 0 0 0 0 0 1004.0 h 4.0",
    ]
    # no PARAM: the guessed increments and ranges of GuessAngleIncrement / GuessAngleRange
    lines_b = []
    for n in (181, 180, 361, 360, 401, 400, 90):
        lines_b.append(f"FLASER {n} " + nums(rng.uniform(0.05, 15.0, n)) + " 0 0 0 1 1 0.5 10.0 h 1.0")
        lines_b.append(f"LASER3 {n} " + nums(rng.uniform(0.05, 15.0, n)))
    # numbers in forms std::istream reads specially
    lines_c = [
        "ODOM 1e-3 -0.0 +2.5 .5 5. 0x10 7 h 1",
        "ODOM 1.0 2.0",
        "ODOM abc 2.0 3.0 4 5 6 7 h 8",
        "RAWLASER2 0 -1 2 0.5 10 0.01 0 3 1.25 nan 2.5 0 1005 h 5",
    ]
    return ["\n".join(lines_a) + "\n", "\n".join(lines_b) + "\n", "\n".join(lines_c)]


def ref_load(L, text):
    n = C.c_int()
    raw = text.encode()
    need = L.ref_carmen_load(raw, None, 0, None, 0, C.byref(n))
    out = np.zeros(max(1, need))
    ids = C.create_string_buffer(64 * (n.value + 1) + 1024)
    L.ref_carmen_load(raw, out.ctypes.data_as(C.POINTER(C.c_double)), need, ids, len(ids), C.byref(n))
    return out[:need], [s.decode() for s in ids.raw.split(b"\0")[: n.value]], n.value


def load_ref_lib():
    L = C.CDLL(REF_SO)
    L.ref_carmen_load.restype = C.c_longlong
    L.ref_carmen_load.argtypes = [C.c_char_p, C.POINTER(C.c_double), C.c_longlong, C.c_char_p, C.c_longlong,
                                  C.POINTER(C.c_int)]
    return L


def main():
    L = load_ref_lib()
    cases = []
    for text in carmen_texts():
        stream, ids, nrec = ref_load(L, text)
        cases.append(dict(text=text, stream=[float(x).hex() for x in stream], ids=ids, records=nrec))
    json.dump(dict(source="reference CarmenLogReader::Load via oracle/_ref/libref_pin.so", cases=cases),
              open(OUT, "w"), indent=0)
    print(f"wrote {OUT}: {len(cases)} cases")


if __name__ == "__main__":
    main()
