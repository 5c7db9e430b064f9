// psgd_libsvm.cpp -- LIBSVM text ingest into CSR partitions (the caller side of the hot path:
// MLUtils.loadLibSVMFile(sc, path, numFeatures, minPartitions) [ext Spark MLlib 1.6.1] feeding
// the RDD that ParallelizedSGD.runParallelizedSGD receives, ParallelizedSGD.scala:188).
//
// Partitions follow sc.textFile(path, minPartitions) on a local file [ext Hadoop 2.x
// FileInputFormat / LineRecordReader]: splitSize = max(1, min(totalSize / minPartitions,
// 32 MiB local block)); splits of splitSize while remaining / splitSize > 1.1, then the
// remainder; a line belongs to the split whose (start, end] holds its first byte (offset 0: the
// first split). Each line is trimmed; empty lines and lines starting with '#' are skipped; the
// rest is "label idx:val idx:val ..." split on ' ', 1-based indices converted to 0-based and
// required strictly increasing; numFeatures <= 0 means max index + 1 over the file.
// Splits are parsed in parallel (one host thread per split, up to the hardware threads).
#include "../../include/psgd.h"

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace psgd {
int32_t set_error(int32_t code, const std::string& msg);   // psgd_capi.cpp
}

namespace {

struct SplitOut {
    std::vector<double> labels;
    std::vector<int64_t> row_ptr{0};
    std::vector<int32_t> col;
    std::vector<double> val;
    int32_t max_index = -1;
    std::string err;
};

// String.trim(): strips chars <= ' ' from both ends.
void trim(const char*& b, const char*& e) {
    while (b < e && (unsigned char)*b <= ' ') ++b;
    while (e > b && (unsigned char)e[-1] <= ' ') --e;
}

// java.lang.Double.parseDouble (StringOps.toDouble) [ext JDK FloatingDecimal.readJavaFormatString]:
// trimmed; optional sign; "NaN" or "Infinity" (exact case), or a decimal significand with at
// least one digit ("1.", ".5") and an optional e/E exponent with at least one digit, or a hex
// significand 0x/0X with a mandatory p/P binary exponent; then an optional f/F/d/D suffix and
// nothing else. The value is the correctly rounded double (glibc strtod on the validated text;
// the f/F suffix still yields the double -- parseDouble ignores the suffix's type).
bool parse_double(const char* b, const char* e, double* out) {
    trim(b, e);
    const char* p = b;
    bool neg = false;
    if (p < e && (*p == '+' || *p == '-')) neg = *p++ == '-';
    auto rest_is = [&](const char* word) {
        const size_t k = strlen(word);
        return (size_t)(e - p) == k && memcmp(p, word, k) == 0;
    };
    if (rest_is("NaN")) { *out = NAN; return true; }
    if (rest_is("Infinity")) { *out = neg ? -INFINITY : INFINITY; return true; }
    const char* q = p;
    auto digits = [&](bool hex) {
        const char* s0 = q;
        while (q < e && (hex ? isxdigit((unsigned char)*q) : isdigit((unsigned char)*q))) ++q;
        return (int)(q - s0);
    };
    const bool hex = (e - q) >= 2 && q[0] == '0' && (q[1] == 'x' || q[1] == 'X');
    if (hex) q += 2;
    int nd = digits(hex);
    if (q < e && *q == '.') { ++q; nd += digits(hex); }
    if (nd == 0) return false;
    if (hex) {
        if (!(q < e && (*q == 'p' || *q == 'P'))) return false;
        ++q;
        if (q < e && (*q == '+' || *q == '-')) ++q;
        if (digits(false) == 0) return false;
    } else if (q < e && (*q == 'e' || *q == 'E')) {
        ++q;
        if (q < e && (*q == '+' || *q == '-')) ++q;
        if (digits(false) == 0) return false;
    }
    const char* num_end = q;
    if (q < e && (*q == 'f' || *q == 'F' || *q == 'd' || *q == 'D')) ++q;
    if (q != e) return false;
    const std::string s(b, num_end);
    *out = strtod(s.c_str(), nullptr);
    return true;
}

// java.lang.Integer.parseInt (StringOps.toInt): optional sign, one or more decimal digits,
// nothing else (no whitespace), within int range.
bool parse_int(const char* b, const char* e, int64_t* out) {
    const char* p = b;
    bool neg = false;
    if (p < e && (*p == '+' || *p == '-')) neg = *p++ == '-';
    if (p == e) return false;
    int64_t v = 0;
    for (; p < e; ++p) {
        if (!isdigit((unsigned char)*p)) return false;
        v = v * 10 + (*p - '0');
        if (v > (int64_t)INT32_MAX + 1) return false;
    }
    v = neg ? -v : v;
    if (v > INT32_MAX || v < INT32_MIN) return false;
    *out = v;
    return true;
}

void parse_line(const char* b, const char* e, SplitOut& o) {
    trim(b, e);
    if (b == e || *b == '#') return;
    const std::string line(b, e);
    // items = line.split(' '); items.head is the label, the rest non-empty index:value pairs
    const char* p = b;
    const char* q = std::find(p, e, ' ');
    double label;
    if (!parse_double(p, q, &label)) {
        if (o.err.empty()) o.err = "NumberFormatException: bad label in line \"" + line + "\"";
        return;
    }
    int64_t previous = -1;
    std::vector<int32_t> idx;
    std::vector<double> vals;
    p = q;
    while (p < e) {
        ++p;  // the separator
        q = std::find(p, e, ' ');
        if (q > p) {
            const char* c = std::find(p, q, ':');
            int64_t index;
            double value;
            if (c == q || !parse_int(p, c, &index) || !parse_double(c + 1, std::find(c + 1, q, ':'), &value)) {
                if (o.err.empty()) o.err = "NumberFormatException: bad index:value item in line \"" + line + "\"";
                return;
            }
            const int64_t current = index - 1;   // one-based -> zero-based
            if (!(current > previous)) {
                if (o.err.empty())
                    o.err = "requirement failed: indices should be one-based and in ascending order; found current=" +
                            std::to_string(current) + ", previous=" + std::to_string(previous) + "; line=\"" +
                            line + "\"";
                return;
            }
            previous = current;
            idx.push_back((int32_t)current);
            vals.push_back(value);
        }
        p = q;
    }
    o.labels.push_back(label);
    o.col.insert(o.col.end(), idx.begin(), idx.end());
    o.val.insert(o.val.end(), vals.begin(), vals.end());
    o.row_ptr.push_back((int64_t)o.col.size());
    if (!idx.empty()) o.max_index = std::max(o.max_index, idx.back());
}

}  // namespace

extern "C" {

int32_t psgd_libsvm_read(const char* path, int32_t num_features, int32_t min_partitions,
                         psgd_libsvm** out) {
    if (!path || !out) return psgd::set_error(PSGD_EINVAL, "path/out is null");
    *out = nullptr;
    if (min_partitions < 1) return psgd::set_error(PSGD_EINVAL, "requirement failed: minPartitions must be positive");
    FILE* f = fopen(path, "rb");
    if (!f) return psgd::set_error(PSGD_EINVAL, std::string("cannot open ") + path + ": " + strerror(errno));
    std::vector<char> buf;
    {
        fseek(f, 0, SEEK_END);
        const long sz = ftell(f);
        fseek(f, 0, SEEK_SET);
        buf.resize(sz > 0 ? (size_t)sz : 0);
        if (sz > 0 && fread(buf.data(), 1, (size_t)sz, f) != (size_t)sz) {
            fclose(f);
            return psgd::set_error(PSGD_EINVAL, std::string("short read from ") + path);
        }
        fclose(f);
    }
    const int64_t total = (int64_t)buf.size();
    // FileInputFormat.getSplits (one local file)
    const int64_t goal = total / min_partitions;
    const int64_t block = 32LL << 20;
    const int64_t split = std::max<int64_t>(1, std::min(goal, block));
    std::vector<int64_t> starts;
    int64_t rem = total;
    while (split > 0 && (double)rem / (double)split > 1.1) {
        starts.push_back(total - rem);
        rem -= split;
    }
    if (rem != 0 || starts.empty()) starts.push_back(total - rem);
    const int S = (int)starts.size();
    starts.push_back(total);
    // line ownership: a line starting at byte p > 0 belongs to the split with start < p <= end
    std::vector<SplitOut> outs((size_t)S);
    auto work = [&](int s) {
        const int64_t a = starts[(size_t)s], z = starts[(size_t)s + 1];
        int64_t pos = a;
        if (a != 0) {
            // LineRecordReader skips to the first line starting after `a` (a line starting
            // exactly at `a` went to the previous split)
            const char* nl = (const char*)memchr(buf.data() + a, '\n', (size_t)(total - a));
            pos = nl ? (nl - buf.data()) + 1 : total;
        }
        // read every line that starts at pos <= z
        while (pos < total && pos <= z) {
            const char* lb = buf.data() + pos;
            const char* nl = (const char*)memchr(lb, '\n', (size_t)(total - pos));
            const char* le = nl ? nl : buf.data() + total;
            const char* lend = le;
            if (lend > lb && lend[-1] == '\r') --lend;
            parse_line(lb, lend, outs[(size_t)s]);
            if (!outs[(size_t)s].err.empty()) return;
            pos = (le - buf.data()) + 1;
        }
    };
    if (S == 1) {
        work(0);
    } else {
        const int T = std::max(1, std::min<int>(S, (int)std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] { for (int s = t; s < S; s += T) work(s); });
        for (auto& x : th) x.join();
    }
    for (auto& o : outs)
        if (!o.err.empty()) return psgd::set_error(PSGD_EINVAL, o.err);
    int64_t n = 0, nnz = 0;
    int32_t max_index = -1;
    for (auto& o : outs) {
        n += (int64_t)o.labels.size();
        nnz += (int64_t)o.col.size();
        max_index = std::max(max_index, o.max_index);
    }
    // numFeatures <= 0: indices.lastOption.getOrElse(0) reduced with max, + 1
    const int32_t d = num_features > 0 ? num_features : std::max<int32_t>(max_index, 0) + 1;
    if (max_index >= d) {
        return psgd::set_error(PSGD_EINVAL, "requirement failed: index " + std::to_string(max_index) +
                                                " out of bounds for numFeatures " + std::to_string(d));
    }
    psgd_libsvm* r = (psgd_libsvm*)calloc(1, sizeof(psgd_libsvm));
    if (!r) return psgd::set_error(PSGD_ENOMEM, "out of host memory");
    r->n_rows = n;
    r->d = d;
    r->n_parts = S;
    r->part_offsets = (int64_t*)malloc(sizeof(int64_t) * (size_t)(S + 1));
    r->labels = (double*)malloc(sizeof(double) * (size_t)std::max<int64_t>(n, 1));
    r->row_ptr = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
    r->col = (int32_t*)malloc(sizeof(int32_t) * (size_t)std::max<int64_t>(nnz, 1));
    r->val = (double*)malloc(sizeof(double) * (size_t)std::max<int64_t>(nnz, 1));
    if (!r->part_offsets || !r->labels || !r->row_ptr || !r->col || !r->val) {
        psgd_libsvm_free(r);
        return psgd::set_error(PSGD_ENOMEM, "out of host memory");
    }
    int64_t row = 0, ent = 0;
    r->row_ptr[0] = 0;
    for (int s = 0; s < S; ++s) {
        const SplitOut& o = outs[(size_t)s];
        r->part_offsets[s] = row;
        std::copy(o.labels.begin(), o.labels.end(), r->labels + row);
        std::copy(o.col.begin(), o.col.end(), r->col + ent);
        std::copy(o.val.begin(), o.val.end(), r->val + ent);
        for (size_t i = 1; i < o.row_ptr.size(); ++i) r->row_ptr[row + (int64_t)i] = ent + o.row_ptr[i];
        row += (int64_t)o.labels.size();
        ent += (int64_t)o.col.size();
    }
    r->part_offsets[S] = row;
    *out = r;
    return PSGD_OK;
}

void psgd_libsvm_free(psgd_libsvm* r) {
    if (!r) return;
    free(r->part_offsets);
    free(r->labels);
    free(r->row_ptr);
    free(r->col);
    free(r->val);
    free(r);
}

}  // extern "C"
