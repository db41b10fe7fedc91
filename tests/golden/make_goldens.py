"""Extract the reference's own golden vectors into JSON fixtures.

Run once in a container that has /root/reference mounted; the outputs
(`reference_goldens.json`, `dense_input.csv`) are committed so that nothing
at test time reads /root/reference.

Sources (all data, no code):
  TsneHelpersTestSuite.scala:331-348  knnInput / knnResults
  TsneHelpersTestSuite.scala:352-383  densePairwiseAffinitiesResults (perplexity 2, k=10)
  TsneHelpersTestSuite.scala:385-416  denseJointProbabilitiesResults
  TsneHelpersTestSuite.scala:418      denseSumQ
  TsneHelpersTestSuite.scala:420-451  denseUnnormLowDimAffinitiesResults
  TsneHelpersTestSuite.scala:453-464  initialEmbedding
  TsneHelpersTestSuite.scala:466-477  denseGradientResults (theta = 0)
  TsneHelpersTestSuite.scala:479-503  gradientWithMomentumAndGainResults / updatedGainsResults
  TsneHelpersTestSuite.scala:505-529  updatedEmbeddingResults / updatedAndCentredEmbeddingResults
  TsneHelpersTestSuite.scala:531-541  centeringInput / centeringResults
  TsneHelpersTestSuite.scala:543-563  sparse pairwise / joint (C++ implementation, 6 digits)
  src/test/resources/dense_input.csv  10 points x 784 dims, COO (i,j,v)
"""
import json
import re
import shutil
import sys
from pathlib import Path

REF = Path("/root/reference/src/test")
SUITE = REF / "scala" / "TsneHelpersTestSuite.scala"
OUT = Path(__file__).resolve().parent

NUM = r"[-+]?\d+(?:\.\d+)?(?:[eE][-+]?\d+)?"


def block(text, name):
    m = re.search(r"val\s+" + name + r"\b[^=]*=\s*(List\(.*?\n\s*\)(?:\.toSeq)?)", text, re.S)
    if not m:
        raise KeyError(name)
    return m.group(1)


def triples(text, name):
    body = block(text, name)
    return [[int(a), int(b), float(c)] for a, b, c in
            re.findall(r"\(\s*(\d+)\s*,\s*(\d+)\s*,\s*(" + NUM + r")\s*\)", body)]


def dense_vectors(text, name):
    body = block(text, name)
    out = []
    for idx, vals in re.findall(r"\(\s*(\d+)\s*,\s*DenseVector\(([^)]*)\)\s*\)", body):
        out.append([int(idx), [float(v) for v in vals.split(",")]])
    return out


def sparse_vectors(text, name):
    body = block(text, name)
    out = []
    for idx, length, entries in re.findall(
            r"\(\s*(\d+)\s*,\s*SparseVector\((\d+)\)\(([^)]*)\)\s*\)", body):
        vec = [0.0] * int(length)
        for k, v in re.findall(r"(\d+)\s*->\s*(" + NUM + r")", entries):
            vec[int(k)] = float(v)
        out.append([int(idx), vec])
    return out


def main():
    text = SUITE.read_text()
    g = {
        "_source": "TsneHelpersTestSuite.scala (ChristophAl/tsne-flink); extracted by make_goldens.py",
        "knnInput": sparse_vectors(text, "knnInput"),
        "knnResults": triples(text, "knnResults"),
        "densePairwiseAffinitiesResults": triples(text, "densePairwiseAffinitiesResults"),
        "denseJointProbabilitiesResults": triples(text, "denseJointProbabilitiesResults"),
        "denseUnnormLowDimAffinitiesResults": triples(text, "denseUnnormLowDimAffinitiesResults"),
        "initialEmbedding": dense_vectors(text, "initialEmbedding"),
        "denseGradientResults": dense_vectors(text, "denseGradientResults"),
        "gradientWithMomentumAndGainResults": dense_vectors(text, "gradientWithMomentumAndGainResults"),
        "updatedGainsResults": dense_vectors(text, "updatedGainsResults"),
        "updatedEmbeddingResults": dense_vectors(text, "updatedEmbeddingResults"),
        "updatedAndCentredEmbeddingResults": dense_vectors(text, "updatedAndCentredEmbeddingResults"),
        "centeringInput": sparse_vectors(text, "centeringInput"),
        "centeringResults": sparse_vectors(text, "centeringResults"),
        "sparsePairwiseAffinitiesResults": triples(text, "sparsePairwiseAffinitiesResults"),
        "sparseJointProbabilitiesResults": triples(text, "sparseJointProbabilitiesResults"),
    }
    m = re.search(r"val\s+denseSumQ\s*=\s*(" + NUM + ")", text)
    g["denseSumQ"] = float(m.group(1))
    # test parameters as stated in the suite
    g["params"] = {
        "knn": {"k": 2, "metric": "sqeuclidean", "line": "TsneHelpersTestSuite.scala:29-42"},
        "pairwise": {"perplexity": 2.0, "neighbors": 10, "dimension": 784,
                     "line": "TsneHelpersTestSuite.scala:76-98", "tol": 1e-12},
        "jointDense": {"tol": 1e-12, "line": "TsneHelpersTestSuite.scala:100-117"},
        "jointSparse": {"tol": 1e-6, "sumTol": 1e-12, "line": "TsneHelpersTestSuite.scala:119-137"},
        "gradient": {"theta": 0.0, "metric": "sqeuclidean", "tol": 1e-12,
                     "line": "TsneHelpersTestSuite.scala:168-209"},
        "update": {"minGain": 0.01, "momentum": 0.5, "learningRate": 300.0, "tol": 1e-9,
                   "line": "TsneHelpersTestSuite.scala:233-271"},
        "iteration": {"momentum": 0.5, "learningRate": 300.0, "theta": 0.0, "tol": 1e-9,
                      "line": "TsneHelpersTestSuite.scala:273-327"},
    }
    for key, want in [("knnResults", 18), ("densePairwiseAffinitiesResults", 90),
                      ("denseJointProbabilitiesResults", 90), ("initialEmbedding", 10),
                      ("denseGradientResults", 10), ("sparsePairwiseAffinitiesResults", 24),
                      ("sparseJointProbabilitiesResults", 32), ("knnInput", 9)]:
        if len(g[key]) != want:
            sys.exit(f"{key}: expected {want} entries, got {len(g[key])}")
    (OUT / "reference_goldens.json").write_text(json.dumps(g, indent=1))
    shutil.copyfile(REF / "resources" / "dense_input.csv", OUT / "dense_input.csv")
    print("wrote", OUT / "reference_goldens.json")


if __name__ == "__main__":
    main()
