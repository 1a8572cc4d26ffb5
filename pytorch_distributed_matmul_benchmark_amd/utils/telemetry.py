"""GPU counting without HIP, and clock / power sampling during a timed region.

``visible_gpus()`` answers "how many GPUs can this process's ranks use?"
from sysfs (the KFD topology: nodes with SIMDs whose DRM render node this
process may open) and the ``*_VISIBLE_DEVICES`` lists — never through HIP,
so a launcher can ask before any process touches the GPU (bench.py's
self-launch parent; forking ranks after HIP initialised is unsafe).

``ClockSampler`` polls amdsmi (GFX clock MHz, socket power W) from a
background thread while a benchmark mode runs, so a JSON line says which
clock each number was measured at: on MI355X random-data bf16 GEMMs are
power-bound (1.69-1.75 GHz at ~1.4 kW), and a mode measured after a long
one can run on a hotter, slower chip (VERDICT r2 "thermal drift").
"""
from __future__ import annotations

import glob
import os
import threading
from typing import List, Optional


def _env_list(name: str) -> Optional[List[str]]:
    v = os.environ.get(name)
    if v is None:
        return None
    return [x for x in (s.strip() for s in v.split(",")) if x != ""]


def sysfs_gpus() -> int:
    """GPUs in the KFD topology whose render node this process can open."""
    n = 0
    for props in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            kv = dict(line.split(None, 1) for line in open(props).read().splitlines() if " " in line)
        except OSError:
            continue
        if int(kv.get("simd_count", "0")) <= 0:
            continue  # a CPU node
        minor = kv.get("drm_render_minor")
        if minor is not None and not os.access(f"/dev/dri/renderD{int(minor)}", os.R_OK | os.W_OK):
            continue
        n += 1
    return n


def amdsmi_gpus() -> int:
    try:
        import amdsmi

        amdsmi.amdsmi_init()
        try:
            return len(amdsmi.amdsmi_get_processor_handles())
        finally:
            amdsmi.amdsmi_shut_down()
    except Exception:
        return 0


def visible_gpus() -> int:
    """GPUs the ranks of this job may use, without initialising HIP."""
    n = sysfs_gpus() or amdsmi_gpus()
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        lst = _env_list(var)
        if lst is not None:
            n = min(n, len(lst)) if n else len(lst)
    return n


class ClockSampler:
    """Median GFX clock (MHz) and socket power (W) of one GPU while active,
    polled every ``period_s`` (5 ms: a 0.1 s timed region still gets ~20
    samples), with the sample counts — a median of a handful of samples is
    reported as such, and a region shorter than the sensor's own averaging
    window (the socket-power reading lags by tens of ms) shows it in
    ``power_key``.

    ``with ClockSampler(device) as s: ...`` then ``s.result()`` ->
    ``{"sclk_mhz", "power_w", "sclk_samples", "power_samples", "power_key"}``
    (values None when amdsmi is unavailable or the device cannot be matched)."""

    def __init__(self, device, period_s: float = 0.005):
        self.device = device
        self.period = period_s
        self._clk: List[float] = []
        self._pwr: List[float] = []
        self._pkey: Optional[str] = None
        self._stop = threading.Event()
        self._t = None
        self._h = None
        self._smi = None

    def _handle(self):
        import amdsmi
        import torch

        amdsmi.amdsmi_init()
        self._smi = amdsmi
        props = torch.cuda.get_device_properties(self.device)
        want = (getattr(props, "pci_domain_id", 0), getattr(props, "pci_bus_id", -1),
                getattr(props, "pci_device_id", -1))
        for h in amdsmi.amdsmi_get_processor_handles():
            bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # "dddd:bb:dd.f"
            dom, bus, df = bdf.split(":")
            if (int(dom, 16), int(bus, 16), int(df.split(".")[0], 16)) == want:
                return h
        return None

    def _run(self):
        amdsmi = self._smi
        while not self._stop.is_set():
            try:
                c = amdsmi.amdsmi_get_clock_info(self._h, amdsmi.AmdSmiClkType.GFX)
                v = c.get("clk", c.get("cur_clk"))
                if isinstance(v, (int, float)) and v > 0:
                    self._clk.append(float(v))
                p = amdsmi.amdsmi_get_power_info(self._h)
                for key in ("current_socket_power", "average_socket_power", "socket_power"):
                    w = p.get(key)
                    if isinstance(w, (int, float)) and w > 0:
                        self._pwr.append(float(w))
                        self._pkey = key
                        break
            except Exception:
                pass
            self._stop.wait(self.period)

    def __enter__(self):
        if getattr(self.device, "type", "cpu") == "cuda":
            try:
                self._h = self._handle()
            except Exception:
                self._h = None
            if self._h is not None:
                self._t = threading.Thread(target=self._run, daemon=True)
                self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=2.0)
        if self._smi is not None:
            try:
                self._smi.amdsmi_shut_down()
            except Exception:
                pass
        return False

    def result(self) -> dict:
        def median(xs):
            if not xs:
                return None
            v = sorted(xs)
            h = len(v) // 2
            return round(v[h] if len(v) % 2 else 0.5 * (v[h - 1] + v[h]), 1)
        return {"sclk_mhz": median(self._clk), "power_w": median(self._pwr),
                "sclk_samples": len(self._clk), "power_samples": len(self._pwr),
                "power_key": self._pkey}

