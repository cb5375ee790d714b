"""GPU clock / power / temperature sampled over a timed window.

The same tree runs 1-3 % apart on different MI355X boxes, and the driver's box has been slower than
the builder's: the MFMA-dense step holds a DVFS clock well under 2.4 GHz (``MI355X_MICROARCH.md``
"DVFS give-back"), so a benchmark line that carries the clock, board power and junction temperature
it ran at can explain such a gap instead of leaving it as noise. A daemon thread polls amdsmi
(through ``torch.cuda.clock_rate`` / ``power_draw`` / ``temperature``, which map the HIP device
index to the amdsmi handle) every ``interval_s`` while the timed steps run; the host thread only
launches kernels there, so the poll costs the step nothing measurable (~1 ms of host time per
sample). Any failure (no amdsmi, a CPU run) is reported in the block instead of raised.
"""

from __future__ import annotations

import statistics
import threading
import time


def _stats(xs: list[float]) -> dict:
    if not xs:
        return {}
    return {"min": round(min(xs), 1), "median": round(statistics.median(xs), 1), "mean": round(statistics.fmean(xs), 1),
            "max": round(max(xs), 1)}


class GpuSampler:
    """``with GpuSampler(device) as s: ...`` then ``s.summary()`` -> the JSON ``gpu_clocks`` block."""

    def __init__(self, device, interval_s: float = 0.25):
        self.device = device
        self.interval_s = interval_s
        self.sclk: list[float] = []
        self.power: list[float] = []
        self.temp: list[float] = []
        self.error: str | None = None
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self._t0 = self._t1 = 0.0

    def _sample(self) -> None:
        import torch

        self.sclk.append(float(torch.cuda.clock_rate(self.device)))
        self.power.append(float(torch.cuda.power_draw(self.device)))
        self.temp.append(float(torch.cuda.temperature(self.device)))

    def _run(self) -> None:
        while not self._stop.is_set():
            try:
                self._sample()
            except Exception as e:  # noqa: BLE001 - diagnostics never fail the benchmark
                self.error = f"{type(e).__name__}: {e}"[:200]
                return
            self._stop.wait(self.interval_s)

    def __enter__(self) -> "GpuSampler":
        if getattr(self.device, "type", "cpu") != "cuda":
            self.error = "not a GPU run"
            return self
        self._t0 = time.perf_counter()
        self._thread = threading.Thread(target=self._run, name="gpu-sampler", daemon=True)
        self._thread.start()
        return self

    def __exit__(self, *exc) -> None:
        self._t1 = time.perf_counter()
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5.0)

    def summary(self) -> dict:
        out: dict = {"source": "amdsmi via torch.cuda.clock_rate/power_draw/temperature", "interval_s": self.interval_s,
                     "samples": len(self.sclk)}
        if self.sclk:
            out["window_s"] = round(self._t1 - self._t0, 2)
            out["sclk_mhz"] = _stats(self.sclk)
            out["power_w"] = _stats(self.power)
            out["temp_junction_c"] = _stats(self.temp)
        if self.error:
            out["error"] = self.error
        try:  # the board's power cap, once (W)
            import amdsmi
            import torch

            h = torch.cuda._get_amdsmi_handler(self.device)
            cap = amdsmi.amdsmi_get_power_cap_info(h).get("power_cap")
            if isinstance(cap, (int, float)):
                out["power_cap_w"] = round(cap / 1e6, 1) if cap > 1e5 else cap  # reported in uW
        except Exception:  # noqa: BLE001
            pass
        return out
