"""The committed evidence bench.py reads (profiles/r*/traffic.json) parses for
every config it can be run on, and each rocprof kernel summary under
profiles/ names kernels that exist in the built library."""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_traffic_file_is_used_only_for_its_own_sources():
    """bench.py's roofline.traffic comes from the latest committed PMC summary
    only when that summary was measured on the same kernel sources (its
    source_digest); otherwise the field is null with the reason."""
    sys.path.insert(0, ROOT)
    import bench
    path = bench.latest_traffic_file()
    assert path, "no profiles/r*/traffic.json"
    doc = json.load(open(path))
    for cfg in ("cfg3a", "cfg3b", "cfg2", "cfg1", "cfg5"):
        t, why = bench.measured_traffic(path, cfg, 10_000_000)
        if doc.get("source_digest") == bench.source_digest() and cfg in doc:
            assert isinstance(t, int) and t > 0, (cfg, t, why)
        else:
            assert t is None and why, (cfg, t)


def test_default_profile_matches_default_kernel():
    """default_bench_kernel_stats.csv of the latest round that has one holds
    the kernel the default bench line names (roofline.kernel)."""
    from hyperdex_amd import synth
    from hyperdex_amd.hashing import kernel_for
    rnd = sorted(os.path.dirname(p) for p in
                 glob.glob(os.path.join(ROOT, "profiles", "r*", "default_bench_kernel_stats.csv")))[-1]
    stats = open(os.path.join(rnd, "default_bench_kernel_stats.csv")).read()
    _, name = kernel_for([r.type for r in synth.CONFIGS["cfg3a"]], 10_000_000)
    assert '"%s"' % name in stats, name
    line = json.load(open(os.path.join(rnd, "default_bench_under_rocprof.json")))
    assert line["roofline"]["kernel"] == name


def test_pmc_record_per_store_schema():
    """Config 5's PMC records are config-3b objects: a bench line over another
    store schema (w200, w1000) gets no traffic of theirs."""
    import bench
    assert bench.pmc_key("cfg3b") == "cfg3b"
    assert bench.pmc_key("cfg5", "keycol") == "cfg5k"
    assert bench.pmc_key("cfg5", "records") == "cfg5r"
    assert bench.pmc_key("cfg5", "columns") == "cfg5"
    key = bench.pmc_key("cfg5", "keycol", "w200")
    assert key == "cfg5k_w200"
    t, why = bench.measured_traffic(bench.latest_traffic_file(), key, 200_000)
    assert t is None and "no PMC record" in why
