"""The CPU baseline's thread count comes from the cgroup CPU quota: on the GPU pool a process
sees every CPU of the host in its affinity mask but may use about 16, and timing torch at 256 threads measured
oversubscription, not the host.  bench.cgroup_cpu_quota reads cgroup v2 cpu.max or v1 cfs_quota/period along the
process's cgroup path (the smallest quota wins)."""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _w(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


def test_v2_quota_smallest_along_the_path(tmp_path):
    root = tmp_path / "cg"
    _w(str(root / "cpu.max"), "max 100000\n")
    _w(str(root / "pod" / "cpu.max"), "3200000 100000\n")
    _w(str(root / "pod" / "job" / "cpu.max"), "1600000 100000\n")
    _w(str(tmp_path / "self"), "0::/pod/job\n")
    cpus, src = bench.cgroup_cpu_quota(str(root), str(tmp_path / "self"))
    assert cpus == pytest.approx(16.0) and src.endswith(os.path.join("job", "cpu.max"))


def test_v2_no_quota(tmp_path):
    root = tmp_path / "cg"
    _w(str(root / "cpu.max"), "max 100000\n")
    _w(str(tmp_path / "self"), "0::/\n")
    assert bench.cgroup_cpu_quota(str(root), str(tmp_path / "self")) is None


def test_v1_quota(tmp_path):
    root = tmp_path / "cg"
    _w(str(root / "cpu,cpuacct" / "docker" / "abc" / "cpu.cfs_quota_us"), "1550000\n")
    _w(str(root / "cpu,cpuacct" / "docker" / "abc" / "cpu.cfs_period_us"), "100000\n")
    _w(str(root / "cpu,cpuacct" / "cpu.cfs_quota_us"), "-1\n")
    _w(str(root / "cpu,cpuacct" / "cpu.cfs_period_us"), "100000\n")
    _w(str(tmp_path / "self"), "4:memory:/docker/abc\n2:cpu,cpuacct:/docker/abc\n0::/\n")
    cpus, src = bench.cgroup_cpu_quota(str(root), str(tmp_path / "self"))
    assert cpus == pytest.approx(15.5) and "abc" in src


def test_baseline_threads_use_the_quota(monkeypatch):
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda *a, **k: (15.5, "/x/cpu.max"))
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(256)))
    threads, cg, src, aff = bench.baseline_threads()
    assert (threads, cg, src, aff) == (16, 15.5, "/x/cpu.max", 256)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(8)))
    assert bench.baseline_threads()[0] == 8  # never more threads than the affinity mask holds


def test_baseline_threads_without_quota(monkeypatch):
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda *a, **k: None)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    assert bench.baseline_threads()[:2] == (16, None)


def test_cpu_baseline_record_has_the_quota(monkeypatch):
    import argparse

    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda *a, **k: (2.0, "/x/cpu.max"))
    args = argparse.Namespace(cpu_sample_params=4096)
    monkeypatch.setattr(bench, "synth_weights", lambda K: [1.0] * K)
    rec = bench.cpu_baseline(args, 4, 4096, 1)
    assert rec["cgroup_cpus"] == 2.0 and rec["cores"] == min(2, rec["affinity_cpus"]) and "full_affinity" not in rec
    assert "cgroup quota" in rec["cores_reason"]
