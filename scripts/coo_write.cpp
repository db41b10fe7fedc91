// coo_write -- raw float64 rows (n x d, little endian) -> the reference's COO
// input (Tsne.readInput, Tsne.scala:138-153): one "i,j,v" line per entry,
// shortest round-trip doubles.  Used to time the native CLI end to end on a
// C3-sized input (scripts/gpu_cli_c3.sh).  usage: coo_write in.bin n d out.csv
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

int main(int argc, char **argv) {
    if (argc != 5) { std::fprintf(stderr, "usage: coo_write in.bin n d out.csv\n"); return 2; }
    const long n = std::atol(argv[2]), d = std::atol(argv[3]);
    std::vector<double> x((size_t)n * d);
    FILE *f = std::fopen(argv[1], "rb");
    if (!f || std::fread(x.data(), sizeof(double), x.size(), f) != x.size()) { std::perror("read"); return 1; }
    std::fclose(f);
    const int T = 16;
    std::vector<std::string> part(T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            std::string &s = part[t];
            const long r0 = n * t / T, r1 = n * (t + 1) / T;
            s.reserve((size_t)(r1 - r0) * d * 28);
            char buf[128];
            for (long i = r0; i < r1; ++i)
                for (long j = 0; j < d; ++j) {
                    auto r = std::to_chars(buf, buf + 96, i);
                    *r.ptr++ = ',';
                    r = std::to_chars(r.ptr, buf + 96, j);
                    *r.ptr++ = ',';
                    r = std::to_chars(r.ptr, buf + 96, x[(size_t)i * d + j]);
                    *r.ptr++ = '\n';
                    s.append(buf, r.ptr);
                }
        });
    for (auto &t : th) t.join();
    FILE *o = std::fopen(argv[4], "wb");
    if (!o) { std::perror("write"); return 1; }
    for (auto &s : part) std::fwrite(s.data(), 1, s.size(), o);
    std::fclose(o);
    return 0;
}
