"""Dev tool: how long torch.cuda.synchronize() returns after the GPU's last kernel ends (the tail
of every timed region), for the HIP runtime's default device schedule and with
hipDeviceScheduleSpin set before the context exists (argv[1] = "spin")."""
import ctypes
import sys
import time

spin = len(sys.argv) > 1 and sys.argv[1] == "spin"
if spin:
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin):", hip.hipSetDeviceFlags(ctypes.c_uint(1)))
import torch  # noqa: E402

torch.cuda.init()
x = torch.zeros(1, device="cuda")
for cycles in (0, 200_000, 2_000_000):
    lat = []
    for _ in range(50):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if cycles:
            torch.cuda._sleep(cycles)
        else:
            x.add_(1)
        e1.record()
        t = time.perf_counter()
        torch.cuda.synchronize()
        host = (time.perf_counter() - t) * 1e6
        lat.append((host, e0.elapsed_time(e1) * 1e3))
    lat.sort()
    h, k = lat[len(lat) // 2]
    print(f"{'spin' if spin else 'default'} sleep {cycles:>8}: sync returns after {h:8.1f} us, "
          f"kernel span {k:8.1f} us (median of 50)")
