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
