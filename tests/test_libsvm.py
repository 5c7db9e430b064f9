"""LIBSVM ingest (psgd_libsvm_read / loadLibSVMFile) against a Python restatement of
MLUtils.loadLibSVMFile [ext Spark MLlib 1.6.1] over sc.textFile(path, minPartitions) on a local
file [ext Hadoop 2.x FileInputFormat.getSplits + LineRecordReader]. CPU only (no device)."""
import numpy as np
import pytest


def hadoop_splits(total, min_partitions, block=32 << 20):
    goal = total // min_partitions
    split = max(1, min(goal, block))
    starts, rem = [], total
    while rem / split > 1.1:
        starts.append(total - rem)
        rem -= split
    if rem != 0 or not starts:
        starts.append(total - rem)
    return starts + [total]


def ref_load(raw: bytes, num_features, min_partitions):
    """Partition p = the lines whose first byte lies in (start_p, end_p] (line 0: split 0)."""
    bounds = hadoop_splits(len(raw), min_partitions)
    line_starts = [0] + [i + 1 for i, c in enumerate(raw) if c == 10 and i + 1 < len(raw)]
    parts = [[] for _ in range(len(bounds) - 1)]
    for ls in line_starts:
        end = raw.find(b"\n", ls)
        line = raw[ls:end if end >= 0 else len(raw)].decode().strip()
        p = 0
        if ls > 0:
            p = next(k for k in range(len(bounds) - 1) if bounds[k] < ls <= bounds[k + 1])
        if not line or line.startswith("#"):
            continue
        items = line.split(" ")
        label = float(items[0])
        idx, val = [], []
        for it in items[1:]:
            if it:
                a, b = it.split(":")[:2]
                idx.append(int(a) - 1)
                val.append(float(b))
        parts[p].append((label, idx, val))
    mx = max([r[1][-1] for ps in parts for r in ps if r[1]] + [0])
    d = num_features if num_features > 0 else mx + 1
    return parts, d


TEXT = (b"# a comment line\n"
        b"1 1:0.5 3:1.25 7:-2\n"
        b"\n"
        b"0  2:1e-3   4:7\r\n"
        b"   1 5:3.5\n"
        b"-1\n"
        b"0 1:1 2:2 3:3 4:4 5:5 6:6 8:8\n"
        b"#trailing comment\n"
        b"1 6:0.25 9:1.5   \n")


@pytest.mark.parametrize("min_parts", [1, 2, 3, 5, 40, 500])
@pytest.mark.parametrize("nf", [-1, 12])
def test_libsvm_matches_restatement(pkg, tmp_path, min_parts, nf):
    f = tmp_path / "data.libsvm"
    f.write_bytes(TEXT)
    data = pkg.loadLibSVMFile(str(f), nf, min_parts)
    parts, d = ref_load(TEXT, nf, min_parts)
    assert len(data.partitions) == len(parts)
    for got, want in zip(data.partitions, parts):
        assert got.d == d
        assert list(got.labels) == [r[0] for r in want]
        assert got.n_rows == len(want)
        for i, (label, idx, val) in enumerate(want):
            a, b = got.row_ptr[i], got.row_ptr[i + 1]
            assert list(got.col[a:b]) == idx
            assert list(got.val[a:b]) == val


def test_libsvm_larger_file_partitions(pkg, tmp_path):
    rng = np.random.default_rng(0)
    lines = []
    for _ in range(3000):
        k = int(rng.integers(0, 12))
        idx = np.sort(rng.choice(500, size=k, replace=False)) + 1
        lines.append(f"{int(rng.integers(0, 2))} " + " ".join(f"{i}:{rng.standard_normal():.6g}" for i in idx))
    raw = ("\n".join(lines) + "\n").encode()
    f = tmp_path / "big.libsvm"
    f.write_bytes(raw)
    for mp in (2, 7, 16):
        data = pkg.loadLibSVMFile(str(f), -1, mp)
        parts, d = ref_load(raw, -1, mp)
        assert [p.n_rows for p in data.partitions] == [len(p) for p in parts]
        assert sum(p.n_rows for p in data.partitions) == 3000
        assert data.partitions[0].d == d


def test_libsvm_errors(pkg, tmp_path):
    f = tmp_path / "bad.libsvm"
    f.write_bytes(b"1 3:1 2:1\n")
    with pytest.raises(pkg.IllegalArgumentException, match="ascending order"):
        pkg.loadLibSVMFile(str(f))
    f.write_bytes(b"1 0:1\n")   # index 0 is not one-based
    with pytest.raises(pkg.IllegalArgumentException, match="ascending order"):
        pkg.loadLibSVMFile(str(f))
    f.write_bytes(b"x 1:1\n")
    with pytest.raises(pkg.IllegalArgumentException, match="NumberFormat"):
        pkg.loadLibSVMFile(str(f))
    f.write_bytes(b"1 5:1\n")
    with pytest.raises(pkg.IllegalArgumentException, match="out of bounds"):
        pkg.loadLibSVMFile(str(f), 3)
    with pytest.raises(pkg.IllegalArgumentException):
        pkg.loadLibSVMFile(str(tmp_path / "missing.libsvm"))


# java.lang.Double.parseDouble's grammar (StringOps.toDouble): accepted forms and their values,
# and forms C's strtod takes that Java rejects
JAVA_DOUBLES_OK = [("1.0d", 1.0), ("2f", 2.0), ("-3.5D", -3.5), ("+4F", 4.0), ("1.", 1.0), (".5", 0.5),
                   ("1e3", 1000.0), ("1E-2", 0.01), ("NaN", float("nan")), ("-Infinity", float("-inf")),
                   ("Infinity", float("inf")), ("0x1.8p1", 3.0), ("0X10P-4d", 1.0), ("-0", -0.0)]
JAVA_DOUBLES_BAD = ["inf", "nan", "infinity", "INFINITY", "1e", "e5", ".", "0x1.8", "1.0dd", "1x", "--1",
                    "0x", "1_0", "1.0e+"]


@pytest.mark.parametrize("text,want", JAVA_DOUBLES_OK)
def test_libsvm_java_double_forms(pkg, tmp_path, text, want):
    f = tmp_path / "ok.libsvm"
    f.write_bytes(f"{text} 2:{text}\n".encode())
    data = pkg.loadLibSVMFile(str(f))
    got_label, got_val = data.partitions[0].labels[0], data.partitions[0].val[0]
    for got in (got_label, got_val):
        if want != want:
            assert got != got
        else:
            assert got == want and np.signbit(got) == np.signbit(want)


@pytest.mark.parametrize("text", JAVA_DOUBLES_BAD)
def test_libsvm_rejects_non_java_doubles(pkg, tmp_path, text):
    f = tmp_path / "bad.libsvm"
    f.write_bytes(f"1 3:{text}\n".encode())
    with pytest.raises(pkg.IllegalArgumentException, match="NumberFormat"):
        pkg.loadLibSVMFile(str(f))
    f.write_bytes(f"{text} 3:1\n".encode())
    with pytest.raises(pkg.IllegalArgumentException, match="NumberFormat"):
        pkg.loadLibSVMFile(str(f))


@pytest.mark.parametrize("text", ["+3", "0003"])
def test_libsvm_java_int_forms(pkg, tmp_path, text):
    f = tmp_path / "ok.libsvm"
    f.write_bytes(f"1 {text}:2.5\n".encode())
    data = pkg.loadLibSVMFile(str(f))
    assert list(data.partitions[0].col) == [2]


@pytest.mark.parametrize("text", ["3.0", "0x3", "2147483648", "1e1", "\t3"])
def test_libsvm_rejects_non_java_ints(pkg, tmp_path, text):
    f = tmp_path / "bad.libsvm"
    f.write_bytes(f"1 {text}:2.5\n".encode())
    with pytest.raises(pkg.IllegalArgumentException, match="NumberFormat"):
        pkg.loadLibSVMFile(str(f))
