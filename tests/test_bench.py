"""bench.py's extras watchdog (CPU): the headline line survives a stalled
secondary timing, and is printed exactly once."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_watchdog_claim_once():
    import bench

    w = bench._ExtrasWatchdog({"value": 1.0}, 0, 30.0)
    assert w.claim() is True
    assert w.claim() is False


def test_watchdog_fires_with_headline_snapshot():
    code = ("import bench, time\n"
            "r = {'metric': 'm', 'value': 2.5}\n"
            "bench._ExtrasWatchdog(r, 0, 0.2)\n"
            "r['late_extra'] = 1\n"  # added after arming: not in the snapshot
            "time.sleep(20)\n"
            "print('not reached')\n")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 0
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and "not reached" not in p.stdout
    d = json.loads(lines[0])
    assert d["value"] == 2.5 and "extras_error" in d and "late_extra" not in d


def test_watchdog_silent_on_other_ranks():
    code = "import bench, time\nbench._ExtrasWatchdog({'value': 1}, 3, 0.2)\ntime.sleep(20)\n"
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 0 and p.stdout.strip() == ""
