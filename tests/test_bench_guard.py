"""bench.py's guard on its one-process extras (host path, device set, CPU
baselines): a failing extra is reported in the line, and one that never
returns has the line printed by the watchdog (CPU only, no GPU needed)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_guarded_reports_an_error():
    sys.path.insert(0, ROOT)
    import bench
    r = {"value": 1.0}

    def boom():
        raise RuntimeError("no device set")
    bench.guarded(r, "config4_device_set", boom)
    assert r["config4_device_set"] == {"error": "RuntimeError: no device set"}
    bench.guarded(r, "secondary", lambda: {"cfg3b": 2})
    assert r["secondary"] == {"cfg3b": 2}


def test_fatal_extra_is_recorded():
    sys.path.insert(0, ROOT)
    import bench
    bench.FAILED_EXTRAS.clear()
    r = {}
    bench.guarded(r, "host_path", lambda: {"GiBps": 1.0}, fatal=True)
    assert bench.FAILED_EXTRAS == []

    def boom():
        raise RuntimeError("exchange failed")
    bench.guarded(r, "config4_device_set", boom, fatal=True)
    bench.guarded(r, "cpu_baseline", boom)  # not fatal
    assert bench.FAILED_EXTRAS == ["config4_device_set"]
    bench.FAILED_EXTRAS.clear()


def test_result_that_beats_the_watchdog_stands():
    # fn returns before the timer fires: its value is kept and the process goes on
    code = ("import sys, time; sys.path.insert(0, %r); import bench; r = {}; "
            "bench.guarded(r, 'host_path', lambda: (time.sleep(0.5), {'ok': 1})[1], watchdog_s=0.7); "
            "time.sleep(1.0); print('after', r['host_path'])" % ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=50)
    assert p.returncode == 0 and "after {'ok': 1}" in p.stdout


def test_watchdog_prints_the_line_and_exits():
    code = ("import sys, time; sys.path.insert(0, %r); import bench; r = {'metric': 'm', 'value': 3.0}; "
            "bench.guarded(r, 'config4_device_set', lambda: time.sleep(60), watchdog_s=1); print('not reached')"
            % ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=50)
    assert p.returncode == 3  # bench.WATCHDOG_EXIT: a hang is not a success
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and "not reached" not in p.stdout
    d = json.loads(lines[0])
    assert d["value"] == 3.0 and "watchdog" in d["config4_device_set"]["error"]
