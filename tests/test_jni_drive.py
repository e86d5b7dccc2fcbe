"""The JNI shim (jni/redisson_sketch_jni.c) driven end to end without a JVM.

jni/sk-jni-drive compiles the shim with a fake JNIEnv (Java arrays as {length, element size, data}) and links the
real libredisson_sketch.so, then calls the SketchNative entry points the Java executors use
(java/org/redisson/gpu/*.java) the way SketchDispatch packs their arguments.  Here its printed results are
checked against the oracle: on CPU the host-only entry points (calcSlot) and the clean "no device" exit; on the
GPU every command of the script.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVE = os.path.join(ROOT, "jni", "sk-jni-drive")


def _run():
    if not os.path.exists(DRIVE):
        pytest.skip("jni/sk-jni-drive not built (make -C jni drive; __graft_entry__.build() builds it)")
    r = subprocess.run([DRIVE], capture_output=True, text=True, timeout=120)
    lines = {}
    for ln in r.stdout.splitlines():
        k, _, v = ln.partition(" ")
        lines[k] = v.split()
    return r.returncode, lines, r


def test_jni_drive_host_entry_points():
    rc, out, r = _run()
    assert out["calcSlot"] == ["11058", "2515", str(__import__("redisson_amd").calc_slot(b"{bf}__config"))]
    assert rc in (0, 77), r.stderr
    if rc == 77:
        assert "NODEVICE" in out


@pytest.mark.gpu
def test_jni_drive_every_entry_point(O):
    rc, out, r = _run()
    assert rc == 0 and "done" in out, r.stdout + r.stderr
    ref = O.HLLStore()
    assert out["pfadd"] == ["0"] + [str(int(x)) for x in ref.pfadd([b"jd:a", b"jd:b", b"jd:a"],
                                                                    [[b"x", b"y"], [b"z"], [b"x"]])]
    assert out["resolve_created"] == ["0", "0", "0"]
    assert out["lookup"] == ["0", "1", "-1"]
    assert out["pfaddIds"] == ["0"] + [str(int(x)) for x in ref.pfadd([b"jd:a", b"jd:b"], [[b"q"], [b"r"]])]
    assert out["pfaddIdsPrefix"] == ["0"] + [str(int(x)) for x in ref.pfadd([b"jd:a", b"jd:b"],
                                                                             [[b"preq2"], [b"prer2"]])]
    ca, cb, cab = ref.count([b"jd:a"]), ref.count([b"jd:b"]), ref.count([b"jd:a", b"jd:b"])
    assert out["pfcount"] == ["0", str(ca), str(cb), str(cab)]
    assert out["pfcountIds"] == ["0", str(ca), str(cb)]
    ref.merge(b"jd:m", [b"jd:a", b"jd:b"])
    assert out["pfmerge_count"] == ["0", str(ref.count([b"jd:m"]))]
    assert out["setbit"] == ["0", "0", "0", "1", "0"]
    assert out["getbit"] == ["0", "0", "1", "1", "0"]
    assert out["void_getbit"] == ["0", "1", "1", "0"]   # SETBIT_VOID with a null reply array
    assert out["bitcount"] == ["0", "1"] and out["strlen"] == ["0", "13"]
    s = bytearray(13)
    s[100 >> 3] |= 0x80 >> (100 & 7)
    t = bytearray(1)
    t[0] |= 0x80 >> 7
    assert out["bitop_or"] == ["0", "13"]
    assert out["get"] == ["0"] + [str(x) for x in O.bitop("OR", [bytes(s), bytes(t)])]
    assert out["get_missing"] == ["1"]
    assert out["set_getbit"] == ["0", "1", "1"]
    assert out["type_hll"] == ["0", "1"]
    assert out["typeMany"] == ["0", "1", "2", "0"]
    assert out["bitsetLength"] == ["0", "101"]
    assert out["bloomTryInit"] == ["0", "1"]
    assert out["bloomConfig"] == ["0", "729", "100", "5", "0.0300"]
    bs = O.BitString(16)
    adds = bs.bloom_add(729, 5, [b'"e1"', b'"e2"', b'"e1"'])
    assert out["bloomAdd"] == ["0"] + [str(int(x)) for x in adds]
    assert out["bloomContains"] == ["0"] + [str(int(x)) for x in bs.bloom_contains(729, 5, [b'"e1"', b'"e3"'])]
    assert out["bloomContains_changed"] == ["-3"]
    assert out["bloomContainsPrefix"] == out["bloomContains"]
    assert out["bloomAddPrefix"] == ["0"] + [str(int(x)) for x in bs.bloom_add(729, 5, [b'"e4"', b'"e5"'])]
    assert out["bloomCount"] == ["0", str(O.bloom_count(729, 5, bs.bitcount()))]  # after the prefix-form adds
    assert out["setBitRange_bitcount"] == ["0", "18"]
    assert out["ticket"] == ["1", "0"]
    assert out["del"] == ["0", "1"]
    assert out["pfaddIds_stale"] == ["-11"]
    assert "not held by a key" in " ".join(out["lastError"])
    assert out["flushall"] == ["0"]
