"""GPU clock / power / temperature state for the bench line (attribute run-to-run swings).

``GpuMonitor(local)`` finds the HIP device's PCI function (torch's ``pci_domain_id`` / ``pci_bus_id`` /
``pci_device_id``) and reads its state, preferring amdsmi's gpu-metrics table (the SMU's own averages: gfx / memory /
fabric clocks, socket power, hotspot and memory temperatures, throttle status, the energy accumulator) and falling
back to sysfs (``pp_dpm_sclk`` / ``pp_dpm_mclk`` / ``pp_dpm_fclk`` current levels, hwmon power and temperatures).
``sample()`` runs a background sampler over a timed region and returns min / median / max per field plus the energy
accumulator's delta.  Every reader is best-effort: a box without amdsmi or sysfs access yields ``{"available":
false, "reason": ...}``, never an exception into the measurement.  Measurement infrastructure, not product code.
"""

from __future__ import annotations

import os
import statistics
import threading
import time

# gpu-metrics fields recorded (amdsmi_get_gpu_metrics_info keys; absent or "N/A" ones are skipped)
METRIC_FIELDS = (
    "average_gfxclk_frequency", "current_gfxclk", "average_uclk_frequency", "current_uclk", "current_socclk",
    "current_fclk", "average_fclk_frequency", "average_socket_power", "current_socket_power",
    "temperature_hotspot", "temperature_mem", "temperature_edge", "average_gfx_activity", "average_umc_activity",
    "throttle_status", "indep_throttle_status",
)


def _num(v):
    if isinstance(v, bool):
        return int(v)
    if isinstance(v, (int, float)):
        return v
    if isinstance(v, str):
        try:
            return float(v.split()[0])
        except (ValueError, IndexError):
            return None
    return None


class GpuMonitor:
    def __init__(self, local: int = 0):
        self.local = int(local)
        self.handle = None
        self.sysfs = None
        self.reason = None
        self._amdsmi = None
        bdf = self._bdf()
        try:
            import amdsmi

            amdsmi.amdsmi_init()
            self._amdsmi = amdsmi
            for h in amdsmi.amdsmi_get_processor_handles():
                if bdf is None or str(amdsmi.amdsmi_get_gpu_device_bdf(h)).lower() == bdf:
                    self.handle = h
                    break
            if self.handle is not None:
                self.snapshot_raw()  # the first read can fail on a box that hides the metrics table
        except Exception as e:  # noqa: BLE001 -- best effort: fall back to sysfs
            self.handle = None
            self.reason = f"amdsmi: {type(e).__name__}: {e}"
        if self.handle is None and bdf is not None:
            d = f"/sys/bus/pci/devices/{bdf}"
            if os.path.isdir(d):
                self.sysfs = d
        self.bdf = bdf

    def _bdf(self):
        try:
            import torch

            p = torch.cuda.get_device_properties(self.local)
            return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        except Exception:  # noqa: BLE001
            return None

    @property
    def available(self) -> bool:
        return self.handle is not None or self.sysfs is not None

    def snapshot_raw(self) -> dict:
        if self.handle is not None:
            m = self._amdsmi.amdsmi_get_gpu_metrics_info(self.handle)
            out = {}
            for k in METRIC_FIELDS:
                v = _num(m.get(k))
                if v is not None:
                    out[k] = v
            gfx = m.get("current_gfxclks")
            if isinstance(gfx, (list, tuple)):
                vals = [x for x in (_num(v) for v in gfx) if x]
                if vals:
                    out["current_gfxclks_min"], out["current_gfxclks_max"] = min(vals), max(vals)
            e = _num(m.get("energy_accumulator"))
            if e is not None:
                out["energy_accumulator"] = e
            return out
        if self.sysfs is not None:
            return self._sysfs_state()
        return {}

    def _sysfs_state(self) -> dict:
        out = {}
        for name in ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk", "pp_dpm_socclk"):
            try:
                with open(os.path.join(self.sysfs, name)) as f:
                    cur = [ln for ln in f.read().splitlines() if ln.rstrip().endswith("*")]
                if cur:
                    out[name + "_mhz"] = _num(cur[0].split(":", 1)[1].strip().lower().replace("mhz", " "))
            except (OSError, IndexError):
                pass
        hw = os.path.join(self.sysfs, "hwmon")
        try:
            for h in os.listdir(hw):
                base = os.path.join(hw, h)
                for fn in os.listdir(base):
                    if fn.startswith(("power", "temp")) and fn.endswith(("_input", "_average")):
                        try:
                            with open(os.path.join(base, fn)) as f:
                                v = float(f.read().strip())
                        except (OSError, ValueError):
                            continue
                        label = fn
                        lab = os.path.join(base, fn.split("_")[0] + "_label")
                        if os.path.exists(lab):
                            with open(lab) as f:
                                label = f"{fn.split('_')[0]}_{f.read().strip()}"
                        out[label] = v / (1e6 if fn.startswith("power") else 1e3)  # W, degrees C
        except OSError:
            pass
        return out

    def snapshot(self) -> dict:
        if not self.available:
            return {"available": False, "reason": self.reason or "no amdsmi handle or sysfs node for this device"}
        try:
            return {"available": True, "source": "amdsmi gpu_metrics" if self.handle is not None else "sysfs",
                    "bdf": self.bdf, **self.snapshot_raw()}
        except Exception as e:  # noqa: BLE001
            return {"available": False, "reason": f"{type(e).__name__}: {e}"}

    def sample(self, interval_s: float = 0.05) -> "_Sampler":
        return _Sampler(self, interval_s)


class _Sampler:
    """``with mon.sample() as s: <timed region>``; then ``s.summary()``."""

    def __init__(self, mon: GpuMonitor, interval_s: float):
        self.mon, self.interval = mon, interval_s
        self.rows, self._stop = [], threading.Event()
        self._t = None
        self.t0 = self.t1 = None

    def _run(self):
        while True:
            try:
                r = self.mon.snapshot_raw()
                r["_t"] = time.perf_counter()
                self.rows.append(r)
            except Exception:  # noqa: BLE001
                pass
            if self._stop.wait(self.interval):
                break

    def __enter__(self):
        self.t0 = time.perf_counter()
        if self.mon.available:
            self._t = threading.Thread(target=self._run, name="gpu-state-sampler", daemon=True)
            self._t.start()
        return self

    def __exit__(self, *exc):
        self.t1 = time.perf_counter()
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=2.0)
        return False

    def summary(self) -> dict:
        if not self.mon.available:
            return {"available": False, "reason": self.mon.reason or "no amdsmi handle or sysfs node"}
        rows = [r for r in self.rows if r]
        out = {"available": True, "source": "amdsmi gpu_metrics" if self.mon.handle is not None else "sysfs",
               "samples": len(rows), "interval_s": self.interval}
        keys = sorted({k for r in rows for k in r if k not in ("energy_accumulator", "_t")})
        for k in keys:
            vals = [r[k] for r in rows if k in r]
            if k in ("throttle_status", "indep_throttle_status"):
                out[k] = sorted({int(v) for v in vals})
            else:
                out[k] = {"min": min(vals), "median": statistics.median(vals), "max": max(vals)}
        en = [(r["_t"], r["energy_accumulator"]) for r in rows if "energy_accumulator" in r]
        if len(en) >= 2 and en[-1][0] > en[0][0]:
            # the SMU's energy counter between the first and the last sample (its unit is the firmware's; the
            # ratio between runs is what compares)
            out["energy_accumulator_delta"] = en[-1][1] - en[0][1]
            out["energy_window_s"] = round(en[-1][0] - en[0][0], 4)
        out["region_s"] = round(self.t1 - self.t0, 4) if self.t1 else None
        return out
