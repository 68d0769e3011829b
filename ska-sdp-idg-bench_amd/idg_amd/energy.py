"""GPU energy over a timed region via amdsmi (the
reference's optional PowerSensor hook, app/HIP/util.cpp:134-159, reports
joules and watts next to its kernel timings; on MI355X the device's own
accumulated-energy counter serves instead).

Usage:
    meter = EnergyMeter(local_rank)   # None-safe: .available tells
    meter.start(); ...timed work...; joules = meter.stop()

Everything degrades to `available = False` (and stop() -> None) when amdsmi
is missing or the counter cannot be read; it never affects the timed path.
"""


def _handle_of(amdsmi, handles, device_index):
    """The amdsmi handle of HIP device `device_index`: matched by PCI
    domain:bus:device (HIP and amdsmi need not enumerate in the same order,
    and HIP_VISIBLE_DEVICES renumbers), else by position."""
    try:
        import torch
        p = torch.cuda.get_device_properties(device_index)
        want = (int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
        for h in handles:
            bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # "dddd:bb:dd.f"
            dom, bus, rest = bdf.split(":")
            if (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)) == want:
                return h
    except Exception:
        pass
    return handles[min(device_index, len(handles) - 1)]


class EnergyMeter:
    def __init__(self, device_index=0):
        self.available = False
        self._smi = None
        self._handle = None
        self._e0 = None
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            handles = amdsmi.amdsmi_get_processor_handles()
            if not handles:
                return
            self._smi = amdsmi
            self._handle = _handle_of(amdsmi, handles, device_index)
            self._read()  # probe once
            self.available = True
        except Exception:
            self.available = False

    def _read(self):
        """Accumulated energy of the device in joules."""
        e = self._smi.amdsmi_get_energy_count(self._handle)
        # {'energy_accumulator': counts, 'counter_resolution': uJ per count}
        acc = e.get("energy_accumulator", e.get("power"))
        res = e.get("counter_resolution", 1.0)
        return float(acc) * float(res) * 1e-6

    def start(self):
        if self.available:
            try:
                self._e0 = self._read()
            except Exception:
                self.available = False

    def stop(self):
        """Joules since start(), or None."""
        if not self.available or self._e0 is None:
            return None
        try:
            return self._read() - self._e0
        except Exception:
            return None

    def power_w(self):
        """Instantaneous socket power in watts, or None."""
        if not self.available:
            return None
        try:
            p = self._smi.amdsmi_get_power_info(self._handle)
            for key in ("current_socket_power", "average_socket_power",
                        "socket_power"):
                v = p.get(key)
                if isinstance(v, (int, float)) and v > 0:
                    return float(v)
        except Exception:
            pass
        return None
