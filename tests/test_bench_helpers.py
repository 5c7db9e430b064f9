"""bench.py's host-side helpers (no GPU): the roofline `traffic` field comes from the committed
rocprofv3 PMC summaries in profiles/, matched to the launched kernel instance."""
import bench


def test_pmc_traffic_matches_committed_profiles():
    t, src = bench.pmc_traffic("c2", "least_squares", 302, "f32", 10_000_000)
    assert src and src.startswith("profiles/") and src.endswith("_c2_pmc.json")
    # HBM bytes per launch within 1 % of the algorithmic (d + 1) * 4 B per row: no re-reads
    assert abs(t / (10_000_000 * 513 * 4) - 1.0) < 0.01
    t3, _ = bench.pmc_traffic("c3", "logistic", 304, "f32", 12_500_000)
    assert abs(t3 / (12_500_000 * 1025 * 4) - 1.0) < 0.01


def test_pmc_traffic_matches_the_updater_instance():
    # c5 runs chain_sparse<float, 0, 1> (Logistic, SquaredL2): ~10 KB of scattered-line traffic
    # per sample (r02 PMC), not the Simple instance
    t, src = bench.pmc_traffic("c5", "logistic", 401, "f32", 20_000_000, updater="squared_l2")
    assert src and src.endswith("_c5_pmc.json")
    assert 5_000 < t / 20_000_000 < 20_000
    assert bench.pmc_traffic("c5", "logistic", 401, "f32", 20_000_000, updater="simple") == (None, None)
    assert bench.pmc_traffic("c2", "least_squares", 302, "f32", 1, updater="adam") == (None, None)


def test_pmc_traffic_none_for_unprofiled_kernels():
    assert bench.pmc_traffic("c1", "logistic", 101, "f64", 100_000) == (None, None)


def test_kernel_labels():
    assert bench.kernel_name(302).startswith("chain_block (NV=2")
    assert bench.kernel_name(411).startswith("chain_sparse_spec")
    assert bench.kernel_name(601).startswith("chain_sparse_lds")
    assert bench.kernel_name(401).startswith("chain_sparse (")
    assert bench.kernel_name(101).startswith("chain_dense")


def test_workloads_cover_the_baseline_configs():
    assert set(bench.WORKLOADS) == {"c1", "c2", "c3", "c4", "c5"}
    grad, n, d, P, step, sdt, _ = bench.WORKLOADS["c2"]
    assert (grad, n, d, P, sdt) == ("least_squares", 10_000_000, 512, 256, "f32")
    assert bench.WORKLOADS["c1"][:4] == ("logistic", 100_000, 100, 4)


def test_fp64_csr_lines_find_their_profiles():
    # c5 in fp64 compute runs chain_sparse64<float, 0, 1> (variant 420): its own PMC summary, not
    # the fp32 chain_sparse one; c4 with the reference's f64 rows runs chain_sparse_lds<double, double, ...>
    t, src = bench.pmc_traffic("c5", "logistic", 420, "f32", 20_000_000, compute="f64", updater="squared_l2")
    assert src and src.endswith("_c5_f64_pmc.json"), src
    assert 5_000 < t / 20_000_000 < 20_000
    t4, src4 = bench.pmc_traffic("c4", "hinge", 620, "f64", 20_000_000, compute="f64")
    assert src4 and src4.endswith("_c4_f64rows_pmc.json"), src4
    assert bench.kernel_name(420).startswith("chain_sparse64")
    assert bench.kernel_name(620).startswith("chain_sparse_lds (fp64")


def test_block64_break_label():
    assert bench.kernel_name(712).endswith("2 chain waves)")
    assert bench.kernel_name(752).endswith("2 chain waves, per-sample isConverged break)")
    assert bench.kernel_name(741).startswith("chain_block64 (NV=1") and "1 chain wave," in bench.kernel_name(741)
    assert bench.kernel_name(342) == "chain_block (NV=2: blocked fp32 chain, 8-row Gram blocks, per-sample isConverged break)"
    assert bench.kernel_name(661).startswith("chain_sparse_lds (fp64") and bench.kernel_name(661).endswith("break)")
    assert bench.kernel_name(641).startswith("chain_sparse_lds (fp32") and "gathered 4" in bench.kernel_name(641)
    assert bench.kernel_name(440).endswith("per sample, per-sample isConverged break)")
    assert bench.kernel_name(461).startswith("chain_sparse64") and bench.kernel_name(461).endswith("break)")
    assert bench.kernel_name(401).endswith("per sample)") and bench.kernel_name(420).endswith("per sample)")


def _fake_record(spec, variant=302):
    """A secondary record shaped as run_workload returns it (after main()'s renames)."""
    wl = spec.split(":")[0]
    return {"spec": spec, "samples_per_s": 1.234567e9, "ms_per_step": 3.1234567, "dtype": "f64",
            "loss": 1.2345e7,
            "config": {"workload": f"{wl}: " + bench.WORKLOADS[wl][6] + " [this run: 20,000,000 rows]",
                       "rows_per_gpu": 20_000_000, "d": 4_194_304, "chains_per_gpu": 1024},
            "roofline": {"bound": "hbm", "achieved": 6543.21, "peak": 8000.0, "unit": "GB/s",
                         "frac": 0.81790123, "frac_step": 0.79123456, "traffic": 2.1e11,
                         "traffic_source": "profiles/r04_c5_f64_pmc.json",
                         "kernel": bench.kernel_name(variant), "bytes_per_launch": 4.8e10,
                         "bytes_per_sample": 2416, "avg_kernel_ms": 94.7169, "avg_epoch_ms": 100.36,
                         "variant": variant, "timing": "HIP events recorded around each chain-kernel launch"},
            "prewarm": {"seconds": 0.5, "epochs": 4}}


def _headline(n_gpus=1):
    rec = _fake_record("c2")
    out = {"metric": "training samples/sec (whole node) + achieved HBM GB/s, logistic SGD 1/2/4/8 GPUs",
           "value": 3.3e9 * n_gpus, "unit": "samples/s", "n_gpus": n_gpus, "steps": 20, "warmup": 5,
           "ms_per_step": 3.1, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f32", "data": "synthetic (device-generated, resident in HBM)",
           "config": rec["config"], "roofline": rec["roofline"], "prewarm": rec["prewarm"]}
    if n_gpus == 1:
        cb = {"value": 1.2e7, "unit": "samples/s", "cores": 16, "kind": "port", "host_cpus": 16,
              "nproc": 256, "sample": "oracle/psgd_oracle.c (fp64 CPU restatement of ParallelizedSGD.scala:"
                                      "243-270 incl. per-sample isConverged; least_squares, simple), 256 "
                                      "partitions x 1024 rows, d=512, 40 epochs, 16 threads, 12.0 s"}
        out["cpu_baseline"] = cb
        out["cpu_baseline_c1"] = dict(cb, sample="oracle/psgd_oracle.c, the whole c1 epoch (100000 x 100 "
                                                 "fp64, 4 partitions, 4 threads = local[4]), 30 epochs, 4.0 s")
    return out


def test_final_line_fits_the_driver_tail(tmp_path, capsys):
    """the 21.7 KB line with 14 full secondaries was not parsed. With the default
    secondaries the printed line is one JSON object under LINE_LIMIT (< 8 KB) that still carries
    the headline, roofline, both cpu baselines and every secondary's summary."""
    import json
    specs = bench.DEFAULT_SECONDARY.split(",")
    assert len(specs) == 14
    records = [_fake_record(s, 420) for s in specs[:-1]] + [{"spec": specs[-1], "error": "RuntimeError: " + "x" * 900}]
    out = _headline()
    out["detail_file"] = bench.write_detail(str(tmp_path / "detail.json"), out, records)
    line = bench.final_line(out, records)
    assert len(line.encode()) < bench.LINE_LIMIT <= 8192
    assert "\n" not in line
    got = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
              "roofline", "cpu_baseline", "cpu_baseline_c1", "secondary_summary"):
        assert k in got, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in got["roofline"], k
    assert [e["spec"] for e in got["secondary_summary"]] == specs
    assert all("frac" in e for e in got["secondary_summary"][:-1])
    assert "secondary" not in got
    # the full records are in the detail file
    detail = json.load(open(tmp_path / "detail.json"))
    assert len(detail["secondary"]) == 14 and detail["secondary"][0]["roofline"]["kernel"]


def test_final_line_multi_gpu():
    import json
    line = bench.final_line(_headline(8), [])
    assert len(line) < bench.LINE_LIMIT
    got = json.loads(line)
    assert got["n_gpus"] == 8 and "secondary_summary" not in got


def test_final_line_multi_gpu_with_baseline_secondaries():
    """at N = 8 the line carries BASELINE's own 8-GPU configs as secondaries
    (c3's 12.5M-row shard per GPU = configs[2], c5's 125M-row shard = configs[4]) with every
    rank's chain-kernel ms and all-gather + fold ms, and stays one parseable line under the cap."""
    import json
    specs = bench.DEFAULT_SECONDARY_MULTI.split(",")
    assert specs[0] == "c3:f32" and "c5:f32" in specs
    assert bench.SECONDARY_ROWS_MULTI["c5"] == 125_000_000 and bench.WORKLOADS["c3"][1] == 12_500_000
    ranks = {"kernel_ms": [7.7354 + i / 1000 for i in range(8)], "xchg_ms": [0.0412 + i / 1e4 for i in range(8)]}
    records = []
    for sp in specs:
        r = _fake_record(sp, 304 if sp.startswith("c3") else 401)
        r["ranks"] = ranks
        if sp.startswith("c5"):
            r["c5_store_probe"] = {"rows_per_chain": 2000, "probe_ms": 12.7094, "marginal_ns_per_row": 3.912,
                                   "mode": "fast"}
        records.append(r)
    out = _headline(8)
    out["ranks"] = ranks
    line = bench.final_line(out, records)
    assert len(line.encode()) < bench.LINE_LIMIT
    got = json.loads(line)
    assert got["n_gpus"] == 8 and len(got["ranks"]["kernel_ms"]) == 8
    assert [e["spec"] for e in got["secondary_summary"]] == specs
    for e in got["secondary_summary"]:
        assert len(e["ranks"]["xchg_ms"]) == 8 and "frac_step" in e
    assert got["secondary_summary"][-1]["c5_store_probe"]["mode"] == "fast"
    assert "frac_step" in got["roofline"]


def test_final_line_shrinks_when_too_long():
    """A line over the limit drops its descriptive strings, never the numbers."""
    import json
    specs = [f"c5:f64:adam:f64" for _ in range(60)]
    line = bench.final_line(_headline(), [_fake_record(s) for s in specs])
    assert len(line) < bench.LINE_LIMIT
    got = json.loads(line)
    assert len(got["secondary_summary"]) == 60
    assert "frac" in got["roofline"] and "value" in got


def test_bench_prints_its_line_last(monkeypatch, capsys, tmp_path):
    """main()'s rank-0 output on stdout is exactly one line (the secondaries do not print)."""
    import inspect
    src = inspect.getsource(bench.main)
    assert src.count("print(") == 1 and "final_line(" in src


def test_arena_carves_aligned_views_and_resets():
    """The one-allocation arena of the synthetic shards (bench.Arena) hands out non-overlapping,
    4 KiB-aligned views of one buffer, refuses to overrun it, and is reused after reset()."""
    import pytest
    import torch
    a = bench.Arena(torch, torch.device("cpu"), bench.shard_bytes("c1"))
    X = a.take((100_000, 100), torch.float64)
    y = a.take((100_000,), torch.float64)
    assert X.shape == (100_000, 100) and y.shape == (100_000,)
    base = a.buf.data_ptr()
    assert (X.data_ptr() - base) % 4096 == 0 and (y.data_ptr() - base) % 4096 == 0
    assert y.data_ptr() >= X.data_ptr() + X.numel() * 8
    X.fill_(1.0)
    y.fill_(2.0)
    assert float(X.sum()) == 1e7 and float(y.sum()) == 2e5
    with pytest.raises(MemoryError):
        a.take((1 << 20,), torch.float64)
    a.reset()
    assert a.take((10,), torch.float32).data_ptr() == X.data_ptr()
    # every default workload fits the arena sized for it
    for spec in bench.DEFAULT_SECONDARY.split(","):
        wl, _, _, sto = (spec.split(":") + ["", "", ""])[:4]
        assert bench.shard_bytes(wl, sto, bench.SECONDARY_ROWS.get(wl, 0)) < 110e9
