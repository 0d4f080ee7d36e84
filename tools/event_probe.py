#!/usr/bin/env python3
"""Can HIP timing events be recorded as nodes of a captured graph here? Tries
hipEventRecordWithFlags(ev, stream, hipEventRecordExternal) inside torch.cuda.graph capture under
each capture_error_mode, replays, and reads hipEventElapsedTime around a known kernel."""
import ctypes

import torch


def main():
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    hip.hipEventRecordWithFlags.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
    hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
    x = torch.randn(4096, 4096, device="cuda")
    for mode in ("thread_local", "global", "relaxed"):
        for flags in (0, 2):  # hipEventDefault, hipEventDisableTiming (control)
            evs = []
            for _ in range(2):
                e = ctypes.c_void_p()
                hip.hipEventCreateWithFlags(ctypes.byref(e), flags)
                evs.append(e)
            s = torch.cuda.Stream()
            g = torch.cuda.CUDAGraph()
            rcs = []
            try:
                with torch.cuda.stream(s):
                    y = x @ x
                    torch.cuda.synchronize()
                    with torch.cuda.graph(g, stream=s, capture_error_mode=mode):
                        rcs.append(hip.hipEventRecordWithFlags(evs[0], ctypes.c_void_p(s.cuda_stream), 1))
                        y = x @ x
                        rcs.append(hip.hipEventRecordWithFlags(evs[1], ctypes.c_void_p(s.cuda_stream), 1))
                    g.replay()
                    torch.cuda.synchronize()
                ms = ctypes.c_float()
                rc = hip.hipEventElapsedTime(ctypes.byref(ms), evs[0], evs[1])
                print(f"mode={mode} flags={flags}: record rcs {rcs}, elapsed rc {rc} = {ms.value:.4f} ms")
            except Exception as e:  # noqa: BLE001
                print(f"mode={mode} flags={flags}: record rcs {rcs}, exception {e!r}, last {hip.hipGetLastError()}")
            hip.hipGetLastError()
            del g


if __name__ == "__main__":
    main()
