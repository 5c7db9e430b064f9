// psgd_run -- a native host driver over the C ABI (include/psgd.h), no Python or torch: the
// caller side a JVM shim would be, in C++. It loads a LIBSVM file the way
// MLUtils.loadLibSVMFile(sc, path, numFeatures, minPartitions) partitions it [ext Spark MLlib
// 1.6.1] (psgd_libsvm_read), registers every partition as CSR rows, and runs the driver loop of
// ParallelizedSGD.runParallelizedSGD (ParallelizedSGD.scala:188-306) around one psgd_run_epoch
// per outer iteration (:238-276). Prints one JSON line: weights, loss history, chain counts.
//
// usage: psgd_run <file.libsvm> [--partitions P] [--features D] [--gradient logistic|
//        least_squares|hinge] [--updater simple|squared_l2|l1|adagrad|adam] [--step S]
//        [--iterations N] [--reg R] [--fraction F] [--tol T] [--compute f64|f32] [--device K]
//        [--checkpoint FILE]
#include "../../include/psgd.h"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

[[noreturn]] void die(const char* what, int32_t rc) {
    std::fprintf(stderr, "psgd_run: %s failed (%d): %s\n", what, rc, psgd_last_error());
    std::exit(rc == PSGD_EINVAL ? 2 : 1);
}

#define CHECK(call)                    \
    do {                               \
        const int32_t rc_ = (call);    \
        if (rc_ != PSGD_OK) die(#call, rc_); \
    } while (0)

int parse_enum(const char* v, const char* const* names, int n, const char* what) {
    for (int i = 0; i < n; ++i)
        if (std::strcmp(v, names[i]) == 0) return i;
    std::fprintf(stderr, "psgd_run: unknown %s '%s'\n", what, v);
    std::exit(2);
}

// breeze.linalg.norm(v, 2) [ext Breeze 0.11]: sqrt of a sequential sum of squares
double norm2(const std::vector<double>& v) {
    double s = 0.0;
    for (double x : v) s += x * x;
    return std::sqrt(s);
}

// java.lang.Math.max (NaN-propagating)
double jmax(double a, double b) {
    if (a != a) return a;
    if (b != b) return b;
    return a >= b ? a : b;
}

// ParallelizedSGD.isConverged (PSGD.scala:324-336)
bool is_converged(const std::vector<double>& prev, const std::vector<double>& cur, double tol) {
    std::vector<double> diff(prev.size());
    for (size_t i = 0; i < prev.size(); ++i) diff[i] = prev[i] - cur[i];
    return norm2(diff) < tol * jmax(norm2(cur), 1.0);
}

void print_array(const char* name, const double* v, size_t n, bool last = false) {
    std::printf("\"%s\": [", name);
    for (size_t i = 0; i < n; ++i) std::printf(i ? ", %.17g" : "%.17g", v[i]);
    std::printf(last ? "]" : "], ");
}

// Checkpoint of the driver loop (--checkpoint FILE; the Python host's DriverCheckpoint): the
// state between iterations -- next iteration, regVal, whether currentWeights is set, converged,
// the loss history and the weights -- behind a fingerprint of the parameters and the data shape
// (numIterations excluded: a finished run can be continued with a larger budget). The fingerprint
// covers the data's shape (rows, partitions, features), not its values: resuming against another
// file of the same shape is the caller's mistake to avoid. Written after every iteration to
// FILE.tmp and renamed over FILE.
struct LoopState {
    int32_t i = 1;
    double regVal = 0.0;
    int32_t have_current = 0, converged = 0;
    std::vector<double> history, weights;
};
constexpr char kCkptMagic[8] = {'P', 'S', 'G', 'D', 'C', 'K', '0', '1'};

std::vector<double> ckpt_fingerprint(const psgd_params& p, int64_t rows, int32_t parts, int32_t d) {
    return {(double)p.gradient, (double)p.updater, (double)p.compute_dtype, p.step_size, p.reg_param,
            p.mini_batch_fraction, p.convergence_tol, p.adam_beta, p.adam_gamma, p.adam_eps,
            (double)p.num_classes, (double)rows, (double)parts, (double)d};
}

bool ckpt_save(const std::string& path, const std::vector<double>& fp, const LoopState& st) {
    const std::string tmp = path + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return false;
    const uint64_t nf = fp.size(), nh = st.history.size(), nw = st.weights.size();
    bool ok = std::fwrite(kCkptMagic, 1, 8, f) == 8 && std::fwrite(&nf, 8, 1, f) == 1 &&
              std::fwrite(fp.data(), 8, nf, f) == nf && std::fwrite(&st.i, 4, 1, f) == 1 &&
              std::fwrite(&st.regVal, 8, 1, f) == 1 && std::fwrite(&st.have_current, 4, 1, f) == 1 &&
              std::fwrite(&st.converged, 4, 1, f) == 1 && std::fwrite(&nh, 8, 1, f) == 1 &&
              std::fwrite(st.history.data(), 8, nh, f) == nh && std::fwrite(&nw, 8, 1, f) == 1 &&
              std::fwrite(st.weights.data(), 8, nw, f) == nw;
    ok = (std::fclose(f) == 0) && ok;
    return ok && std::rename(tmp.c_str(), path.c_str()) == 0;
}

// 1: resumed, 0: no file, -1: unreadable or of other parameters / data
int ckpt_load(const std::string& path, const std::vector<double>& fp, int32_t d, LoopState& st) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return 0;
    char magic[8];
    uint64_t nf = 0, nh = 0, nw = 0;
    std::vector<double> got;
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, kCkptMagic, 8) == 0 &&
              std::fread(&nf, 8, 1, f) == 1 && nf == fp.size();
    if (ok) {
        got.resize(nf);
        ok = std::fread(got.data(), 8, nf, f) == nf && got == fp && std::fread(&st.i, 4, 1, f) == 1 &&
             std::fread(&st.regVal, 8, 1, f) == 1 && std::fread(&st.have_current, 4, 1, f) == 1 &&
             std::fread(&st.converged, 4, 1, f) == 1 && std::fread(&nh, 8, 1, f) == 1 && nh < (1u << 30);
    }
    if (ok) {
        st.history.resize(nh);
        ok = std::fread(st.history.data(), 8, nh, f) == nh && std::fread(&nw, 8, 1, f) == 1 &&
             nw == (uint64_t)d;
    }
    if (ok) {
        st.weights.resize(nw);
        ok = std::fread(st.weights.data(), 8, nw, f) == nw;
    }
    std::fclose(f);
    return ok ? 1 : -1;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <file.libsvm> [options]\n", argv[0]);
        return 2;
    }
    const char* path = argv[1];
    static const char* const kGrad[] = {"logistic", "least_squares", "hinge"};
    static const char* const kUpd[] = {"simple", "squared_l2", "l1", "adagrad", "adam"};
    static const char* const kDt[] = {"f64", "f32"};
    int parts = 2, features = -1, device = 0, iterations = 100;
    std::string checkpoint;
    psgd_params p{};
    p.gradient = PSGD_GRADIENT_LOGISTIC;
    p.updater = PSGD_UPDATER_SIMPLE;
    p.compute_dtype = PSGD_F64;
    p.step_size = 1.0;                 // ParallelizedSGD defaults, PSGD.scala:46-50
    p.reg_param = 0.0;
    p.mini_batch_fraction = 1.0;
    p.convergence_tol = 0.001;
    p.adam_beta = 0.9;                 // AdamSGDUpdater defaults, UPD.scala:241-244
    p.adam_gamma = 0.999;
    p.adam_eps = 1e-8;
    p.num_classes = 2;
    for (int a = 2; a + 1 < argc; a += 2) {
        const std::string k = argv[a];
        const char* v = argv[a + 1];
        if (k == "--partitions") parts = std::atoi(v);
        else if (k == "--features") features = std::atoi(v);
        else if (k == "--device") device = std::atoi(v);
        else if (k == "--iterations") iterations = std::atoi(v);
        else if (k == "--gradient") p.gradient = parse_enum(v, kGrad, 3, "gradient");
        else if (k == "--updater") p.updater = parse_enum(v, kUpd, 5, "updater");
        else if (k == "--compute") p.compute_dtype = parse_enum(v, kDt, 2, "compute dtype");
        else if (k == "--step") p.step_size = std::atof(v);
        else if (k == "--reg") p.reg_param = std::atof(v);
        else if (k == "--fraction") p.mini_batch_fraction = std::atof(v);
        else if (k == "--tol") p.convergence_tol = std::atof(v);
        else if (k == "--checkpoint") checkpoint = v;
        else {
            std::fprintf(stderr, "psgd_run: unknown option %s\n", k.c_str());
            return 2;
        }
    }

    psgd_libsvm* data = nullptr;
    CHECK(psgd_libsvm_read(path, features, parts, &data));
    const int32_t d = data->d;
    psgd_ctx* ctx = nullptr;
    CHECK(psgd_ctx_create(device, &ctx));
    // one registration per partition, as the JVM side does from its mapPartitions tasks
    for (int32_t q = 0; q < data->n_parts; ++q) {
        const int64_t a = data->part_offsets[q], b = data->part_offsets[q + 1];
        CHECK(psgd_register_csr(ctx, q, b - a, d, data->labels + a, data->row_ptr + a, data->col,
                                data->val, PSGD_F64));
    }

    // ParallelizedSGD.runParallelizedSGD, PSGD.scala:188-306 (initialWeights = zeros)
    std::vector<double> weights(d, 0.0), w_new(d);
    std::vector<double> history;
    std::vector<int64_t> counts(data->n_parts);
    std::vector<double> counts_log;
    double epoch_s = 0.0;
    if (p.mini_batch_fraction < 1.0 && p.convergence_tol > 0.0)   // :200-203
        std::fprintf(stderr, "WARN Testing against a convergenceTol when using miniBatchFraction "
                             "< 1.0 can be unstable because of the stochasticity in sampling.\n");
    if (data->n_rows == 0) {                                        // :214-217
        std::fprintf(stderr, "WARN GradientDescent.runMiniBatchSGD returning initial weights, "
                             "no data found\n");
    } else {
        double regVal = 0.0;
        CHECK(psgd_initial_regval(ctx, &p, d, weights.data(), &regVal));   // :231-233
        bool converged = false, have_current = false;
        int first = 1;
        const std::vector<double> fp = ckpt_fingerprint(p, data->n_rows, data->n_parts, d);
        if (!checkpoint.empty()) {
            LoopState st;
            const int r = ckpt_load(checkpoint, fp, d, st);
            if (r < 0) {
                std::fprintf(stderr, "psgd_run: checkpoint %s was written by a run with other parameters "
                                     "or data\n", checkpoint.c_str());
                return 2;
            }
            if (r > 0) {
                first = st.i;
                regVal = st.regVal;
                have_current = st.have_current != 0;
                converged = st.converged != 0;
                history = st.history;
                weights = st.weights;
                std::fprintf(stderr, "WARN resuming at iteration %d from checkpoint %s\n", first, checkpoint.c_str());
            }
        }
        for (int i = first; !converged && i <= iterations; ++i) {          // :237
            p.iteration = i;
            double avgRegVal = 0.0, lossSum = 0.0;
            int64_t batchSize = 0;
            const auto t0 = std::chrono::steady_clock::now();
            CHECK(psgd_run_epoch(ctx, &p, weights.data(), w_new.data(), &avgRegVal, &lossSum,
                                 &batchSize, counts.data()));
            epoch_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            for (int64_t c : counts) counts_log.push_back((double)c);
            if (batchSize > 0) {                                            // :278
                history.push_back(lossSum / (double)batchSize + regVal);   // :283
                regVal = avgRegVal;                                         // :286-287
                if (have_current) converged = is_converged(weights, w_new, p.convergence_tol);
                weights.swap(w_new);
                have_current = true;
            } else {                                                        // :295-297
                std::fprintf(stderr, "WARN Iteration (%d/%d). The size of sampled batch is zero\n",
                             i, iterations);
            }
            if (!checkpoint.empty()) {
                LoopState st;
                st.i = i + 1;
                st.regVal = regVal;
                st.have_current = have_current;
                st.converged = converged;
                st.history = history;
                st.weights = weights;
                if (!ckpt_save(checkpoint, fp, st)) {
                    std::fprintf(stderr, "psgd_run: cannot write checkpoint %s\n", checkpoint.c_str());
                    return 1;
                }
            }
        }
    }
    std::printf("{");
    print_array("weights", weights.data(), weights.size());
    print_array("loss", history.data(), history.size());
    print_array("chain_counts", counts_log.data(), counts_log.size());
    std::printf("\"partitions\": %d, \"rows\": %lld, \"d\": %d, \"epoch_seconds\": %.6f}\n",
                data->n_parts, (long long)data->n_rows, d, epoch_s);
    CHECK(psgd_ctx_destroy(ctx));
    psgd_libsvm_free(data);
    return 0;
}
