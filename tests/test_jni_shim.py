"""The JNI binding a maintainer adds to the Flink job (jni/),
checked as far as this image allows (no JDK, no scalac):

  * the C shim type-checks against include/tsne_hip.h (gcc -fsyntax-only with
    a minimal jni.h stand-in for the few JNIEnv functions it uses);
  * every `native` method of TsneHip.java has its Java_..._TsneHip_<name>
    function in the shim with the same arity (+ env, class);
  * every TsneHip.<name> the Scala bodies call is declared;
  * the Scala bodies keep the reference's TsneHelpers signatures
    (TsneHelpers.scala:41-43, 61-63, 93-95, 162-163, 182, 396-401): metric as
    `(Vector[Double], Vector[Double]) => Double`, no 2 GiB ByteBuffers.
"""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
JNI = ROOT / "jni"


def java_natives():
    text = (JNI / "TsneHip.java").read_text()
    out = {}
    for m in re.finditer(r"public static native \w+(?:\[\])? (\w+)\(([^)]*)\)", text, flags=re.S):
        args = [a for a in m.group(2).split(",") if a.strip()]
        out[m.group(1)] = len(args)
    return out


def test_shim_type_checks_against_c_abi():
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    r = subprocess.run(["gcc", "-fsyntax-only", "-std=c99", "-Wall", "-Wextra", "-Werror",
                        f"-I{JNI / 'jni_stub'}", f"-I{ROOT / 'include'}", str(JNI / "tsne_hip_jni.c")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_every_native_has_its_shim_function():
    natives = java_natives()
    assert len(natives) >= 12
    shim = (JNI / "tsne_hip_jni.c").read_text()
    fns = {}
    for m in re.finditer(r"JNI_FN\((\w+)\)\(([^)]*)\)", shim, flags=re.S):
        fns[m.group(1)] = len([a for a in m.group(2).split(",") if a.strip()])
    assert set(natives) == set(fns), set(natives) ^ set(fns)
    for name, nargs in natives.items():
        assert fns[name] == nargs + 2, name   # JNIEnv *, jclass


def test_scala_bodies_call_declared_natives_with_reference_signatures():
    scala = (JNI / "TsneHipOperators.scala").read_text()
    natives = java_natives()
    for name in set(re.findall(r"TsneHip\.(\w+)\(", scala)):
        assert name in natives, name
    metric = r"metric: \(Vector\[Double\], Vector\[Double\]\) => Double"
    for sig in (rf"def kNearestNeighbors\(input: DataSet\[\(Int, Vector\[Double\]\)\], k: Int,\s+{metric}\)",
                rf"def partitionKnn\(input: DataSet\[\(Int, Vector\[Double\]\)\], k: Int,\s+{metric}, blocks: Int\)",
                rf"def projectKnn\(input: DataSet\[\(Int, Vector\[Double\]\)\], k: Int,\s+{metric}, dimension: Int,"
                r"\s+iterations: Int\)",
                r"def pairwiseAffinities\(input: DataSet\[\(Int, Int, Double\)\], perplexity: Double\)",
                r"def jointDistribution\(input: DataSet\[\(Int, Int, Double\)\]\)",
                rf"learningRate: Double, iterations: Int, {metric},"):
        assert re.search(sig, scala), sig
    assert "allocateDirect" not in scala and "java.nio" not in scala   # off-heap, 64-bit indexes


def test_optimize_rejects_rows_shorter_than_the_point_ids():
    """Tsne.scala:121 sizes each row of P as inputDimension^2 while its indices
    are point ids: the operator refuses a row shorter than the largest id with
    an IllegalArgumentException naming the caller line and INTEGRATION.md 1
    (which documents the one-line caller change)."""
    scala = (JNI / "TsneHipOperators.scala").read_text()
    body = scala[scala.index("def optimize("):]
    m = re.search(r"if \(sv\.length <= maxId\)\s+throw new IllegalArgumentException\(", body)
    assert m, "length check missing in optimize"
    msg = body[m.end():body.index(")\n", m.end())]
    assert "VectorBuilder(number of points)" in msg and "Tsne.scala:121" in msg and "INTEGRATION.md" in msg
    integ = (ROOT / "INTEGRATION.md").read_text()
    assert "new VectorBuilder[Double](numberOfPoints)" in integ
