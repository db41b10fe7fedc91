// tsne_main.cpp -- native CLI with the exact flags and file formats of the
// reference's Tsne.main (Tsne.scala:33-168), running the hot path through
// libtsne_hip on one GPU.  For benchmarking on a box without a JVM/Flink.
//
//   tsne_hip --input X.csv --output Y.csv --dimension D --knnMethod bruteforce
//            [--metric sqeuclidean] [--perplexity 30] [--nComponents 2]
//            [--earlyExaggeration 4] [--learningRate 1000] [--iterations 300]
//            [--randomState 0] [--neighbors 3*perplexity] [--initialMomentum 0.5]
//            [--finalMomentum 0.8] [--theta 0.25] [--loss loss.txt | --lossFile loss.txt]
//            [--knnIterations 3] [--knnBlocks P] [--inputDistanceMatrix] [--executionPlan]
//            [--device 0] [--hostChain]
// The exact kNN methods run kNN -> affinities -> joint -> optimize resident
// in HBM (device_pipeline.hpp); --hostChain (and --knnMethod project, the
// distance-matrix input) take the TsneHelpers mirror, whose operators pass
// host CSR between them as the reference's operators pass DataSets.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "coo_reader.hpp"
#include "device_pipeline.hpp"
#include "tsne_helpers.hpp"

using namespace tsne_flink;

namespace {

// org.apache.flink.api.java.utils.ParameterTool.fromArgs: --key value | --flag
struct Params {
    std::map<std::string, std::string> kv;
    static Params fromArgs(int argc, char **argv) {
        Params p;
        for (int i = 1; i < argc; ++i) {
            std::string a = argv[i];
            if (a.rfind("--", 0) != 0 && a.rfind("-", 0) != 0)
                throw std::invalid_argument("Error parsing arguments '" + a + "'");
            std::string key = a.substr(a.rfind("--", 0) == 0 ? 2 : 1);
            if (i + 1 < argc && std::strncmp(argv[i + 1], "--", 2) != 0) p.kv[key] = argv[++i];
            else p.kv[key] = "__NO_VALUE_KEY";
        }
        return p;
    }
    bool has(const std::string &k) const { return kv.count(k) > 0; }
    std::string getRequired(const std::string &k) const {
        auto it = kv.find(k);
        if (it == kv.end() || it->second == "__NO_VALUE_KEY")
            throw std::runtime_error("No data for required key '" + k + "'");
        return it->second;
    }
    std::string get(const std::string &k, const std::string &def) const {
        auto it = kv.find(k);
        return it == kv.end() ? def : it->second;
    }
    double getDouble(const std::string &k, double def) const { return has(k) ? std::stod(getRequired(k)) : def; }
    // the reference reads these with getLong; accept "4" and (unlike Flink) "4.0"
    long getLong(const std::string &k, long def) const { return has(k) ? (long)std::stod(getRequired(k)) : def; }
};

// Tsne.readDistanceMatrix (Tsne.scala:155-159): raw (i, j, d) triples.
std::vector<Triple> readDistanceMatrix(const std::string &path) {
    const CooTriples t = readCooFile(path);
    std::vector<Triple> out(t.i.size());
    for (size_t e = 0; e < out.size(); ++e) out[e] = {t.i[e], t.j[e], t.v[e]};
    return out;
}

double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

int main(int argc, char **argv) {
    try {
        Params parameters = Params::fromArgs(argc, argv);
        const bool getExecutionPlan = parameters.has("executionPlan");
        const bool inputDistanceMatrix = parameters.has("inputDistanceMatrix");
        const std::string inputPath = parameters.getRequired("input");
        const std::string outputPath = parameters.getRequired("output");
        const int inputDimension = std::stoi(parameters.getRequired("dimension"));
        const std::string metricName = parameters.get("metric", "sqeuclidean");
        const double perplexity = parameters.getDouble("perplexity", 30.0);
        const long nComponents = parameters.getLong("nComponents", 2);
        const double earlyExaggeration = (double)parameters.getLong("earlyExaggeration", 4);
        const double learningRate = parameters.getDouble("learningRate", 1000);
        const long iterations = parameters.getLong("iterations", 300);
        const long randomState = parameters.getLong("randomState", 0);
        const long neighbors = parameters.getLong("neighbors", 3 * (long)perplexity);
        const double initialMomentum = parameters.getDouble("initialMomentum", 0.5);
        const double finalMomentum = parameters.getDouble("finalMomentum", 0.8);
        const double theta = parameters.getDouble("theta", 0.25);
        // the code reads "loss" (Tsne.scala:60); README.md:36 documents "lossFile": accept both
        const std::string lossFile = parameters.get("loss", parameters.get("lossFile", "loss.txt"));
        const std::string knnMethod = parameters.getRequired("knnMethod");
        const int device = (int)parameters.getLong("device", 0);
        const long knnIterations = parameters.getLong("knnIterations", 3);
        (void)parameters.getLong("knnBlocks", 1);

        if (getExecutionPlan) {  // Tsne.scala:89-95: write the plan instead of executing
            std::ofstream pw("tsne_executionPlan.json");
            pw << "{\"nodes\":[{\"id\":1,\"type\":\"source\",\"contents\":\"" << inputPath << "\"},"
               << "{\"id\":2,\"type\":\"knn\",\"contents\":\"" << (inputDistanceMatrix ? "distance-matrix" : knnMethod)
               << " (libtsne_hip)\"},{\"id\":3,\"type\":\"pairwiseAffinities\"},{\"id\":4,\"type\":\"jointDistribution\"},"
               << "{\"id\":5,\"type\":\"optimize\",\"iterations\":" << iterations << "},"
               << "{\"id\":6,\"type\":\"sink\",\"contents\":\"" << outputPath << "\"}]}\n";
            return 0;
        }

        const int32_t metric = getMetric(metricName);  // IllegalArgumentException before any work
        TsneHelpers h(device);
        double t0 = now();
        WorkingSet ws;
        std::map<int32_t, double> loss;
        tsne_params prm;
        tsne_params_default(&prm);
        prm.n_components = (int32_t)nComponents;
        prm.metric = metric;
        prm.learning_rate = learningRate;
        prm.iterations = (int32_t)iterations;
        prm.early_exaggeration = earlyExaggeration;
        prm.initial_momentum = initialMomentum;
        prm.final_momentum = finalMomentum;
        prm.theta = theta;
        // P as CSR over the sorted point ids; the kNN methods keep that form
        // from the GPU's output on (no 10^8-element triple vectors)
        Csr knn;
        bool done = false;
        if (inputDistanceMatrix) {
            knn = toCsr(readDistanceMatrix(inputPath));
        } else {
            // Tsne.readInput's rows, ordered by id as the kNN takes them (readInputDense)
            std::vector<int32_t> ids;
            std::vector<double> X;
            readInputDense(inputPath, inputDimension, ids, X);
            double t1 = now();
            std::fprintf(stderr, "[tsne_hip] read %zu points in %.3f s\n", ids.size(), t1 - t0);
            if (knnMethod != "bruteforce" && knnMethod != "partition" && knnMethod != "project")
                throw std::invalid_argument("Knn method '" + metricName + "' not defined");  // Tsne.scala:78
            if (knnMethod != "project" && ids.size() >= 2 && !parameters.has("hostChain")) {
                // the exact kNN methods: the whole chain resident in HBM (device_pipeline.hpp);
                // --hostChain runs the TsneHelpers mirror's host round trips instead
                DeviceRun run = runOnDevice(h.context(), X, (int64_t)ids.size(), inputDimension, (int32_t)neighbors,
                                            perplexity, prm, randomState);
                std::fprintf(stderr, "[tsne_hip] kNN in %.3f s\n", run.t_knn);
                std::fprintf(stderr, "[tsne_hip] affinities + joint in %.3f s (nnz %lld)\n", run.t_aff,
                             (long long)run.nnz);
                std::fprintf(stderr, "[tsne_hip] %ld iterations in %.3f s\n", iterations, run.t_loop);
                ws.ids = std::move(ids);
                ws.n_components = (int32_t)nComponents;
                ws.y = std::move(run.y);
                loss = std::move(run.loss);
                done = true;
            } else {
                knn = h.kNearestNeighborsCsr(std::move(ids), X, inputDimension, (int32_t)neighbors, metric, knnMethod,
                                             (int32_t)knnIterations, randomState);
                std::fprintf(stderr, "[tsne_hip] kNN in %.3f s\n", now() - t1);
            }
        }
        if (!done) {
            double t2 = now();
            Csr P = h.jointDistributionCsr(h.pairwiseAffinitiesCsr(knn, perplexity));
            {   // the working set's rows are P's non-empty rows (points without an entry drop out)
                bool all = true;
                for (size_t i = 0; i + 1 < P.row_ptr.size(); ++i) all = all && P.row_ptr[i + 1] > P.row_ptr[i];
                if (!all) {
                    const std::vector<Triple> t = fromCsr(P);
                    std::vector<int32_t> ids;
                    for (const auto &e : t)
                        if (ids.empty() || e.i != ids.back()) ids.push_back(e.i);
                    P = toCsr(t, &ids);
                }
            }
            std::fprintf(stderr, "[tsne_hip] affinities + joint in %.3f s (nnz %zu)\n", now() - t2, P.val.size());
            ws = h.initWorkingSet(P.ids, (int32_t)nComponents, randomState);
            double t3 = now();
            h.optimizeCsr(P, ws, learningRate, (int32_t)iterations, metric, earlyExaggeration, initialMomentum,
                          finalMomentum, theta, &loss);
            std::fprintf(stderr, "[tsne_hip] %ld iterations in %.3f s\n", iterations, now() - t3);
        }

        {   // result.map(x => (x._1, x._2(0), x._2(1))).writeAsCsv (Tsne.scala:86);
            // the 3-D extension appends the third component.  Rows formatted
            // by parallel chunks (java.lang.Double.toString each), written in order.
            const size_t nc = (size_t)ws.n_components, rows = ws.ids.size();
            const int T = (int)std::max<size_t>(1, std::min<size_t>(16, rows / 4096));
            std::vector<std::string> part((size_t)T);
            std::vector<std::thread> pool;
            for (int t = 0; t < T; ++t)
                pool.emplace_back([&, t] {
                    std::string &o = part[(size_t)t];
                    for (size_t r = rows * t / T; r < rows * (t + 1) / T; ++r) {
                        o += std::to_string(ws.ids[r]);
                        for (size_t k = 0; k < std::min<size_t>(nc, 3); ++k) {
                            o += ',';
                            o += javaDouble(ws.y[nc * r + k]);
                        }
                        o += '\n';
                    }
                });
            for (auto &th : pool) th.join();
            FILE *f = std::fopen(outputPath.c_str(), "w");
            if (!f) throw std::runtime_error("cannot write " + outputPath);
            for (const std::string &o : part) std::fwrite(o.data(), 1, o.size(), f);
            std::fclose(f);
        }
        std::ofstream lf(lossFile);  // Tsne.scala:99-101
        lf << javaHashMapString(loss);
        std::fprintf(stderr, "[tsne_hip] end-to-end %.3f s\n", now() - t0);
        return 0;
    } catch (const std::invalid_argument &e) {
        std::fprintf(stderr, "java.lang.IllegalArgumentException: %s\n", e.what());
        return 2;
    } catch (const std::exception &e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
}
