// coo_reader.hpp -- the reference's input formats (Tsne.scala:138-159), read
// in parallel from a memory-mapped file.
//
// Tsne.readInput: CSV lines "i,j,v" (Int, Int, Double); row i becomes the
// dense vector x_i with x_i[j] += v (VectorBuilder.add accumulates), rows in
// order of first appearance.  Tsne.readDistanceMatrix: the same lines as raw
// (i, j, d) triples.  The file is split into per-thread byte ranges at line
// boundaries; each thread parses its range (integers by hand, doubles with
// strtod: correctly rounded like java.lang.Double.parseDouble); the triples
// keep file order, so every result is identical to a sequential read.
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace tsne_flink {

struct CooTriples {
    std::vector<int32_t> i, j;
    std::vector<double> v;
};

// Parse "i,j,v" lines of buf[0..len) with `threads` threads (0 = hardware
// concurrency).  Empty lines and a trailing '\r' are accepted; anything else
// malformed throws std::runtime_error naming the line.
CooTriples parseCoo(const char *buf, size_t len, int threads = 0);
// mmap + parseCoo
CooTriples readCooFile(const std::string &path, int threads = 0);
// Tsne.readInput: dense rows (id, x) in order of first appearance; a column
// outside [0, dimension) throws std::out_of_range.
std::vector<std::pair<int32_t, std::vector<double>>> cooToVectors(const CooTriples &t, int dimension);
// Tsne.readInput straight into the kNN's dense form: the distinct ids sorted
// ascending and X (ids.size() x dimension, row-major), x_i[j] the sum of row
// i's values at column j in file order -- the rows of cooToVectors ordered by
// id, without the per-row vectors and the serial passes (the file is parsed,
// its ids marked and its values scattered by `threads` threads; cells that
// occur more than once are re-summed in file order).
void readInputDense(const std::string &path, int dimension, std::vector<int32_t> &ids, std::vector<double> &X,
                    int threads = 0);

}  // namespace tsne_flink
