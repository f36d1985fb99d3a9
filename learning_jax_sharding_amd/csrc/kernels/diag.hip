// Diagnostic kernels (never on a production path).
//
// clock_probe_kernel: the shader clock at one point of the stream, measured -- not read from sysfs
// (MI355X_MICROARCH "DVFS give-back" item 6: the in-kernel clock is delta s_memtime / delta
// s_memrealtime x 100 MHz).  One lane spins until the constant 100 MHz counter has advanced by
// `ticks` and records both deltas; a record per launch, indexed by a device-side counter (a vector
// atomic), so a launch captured into a HIP graph records every replay in order.  bench.py launches
// it after every training step under LJS_CLOCK_PROBE (scripts/clock_ramp.py reads the records
// beside the kernel trace's per-step durations: verdict r5 item 7, the slow start).
#include "common.h"

struct ClockRec {
  unsigned long long d_sclk;   // shader-clock ticks over the spin
  unsigned long long d_ref;    // 100 MHz ticks over the spin
  unsigned long long ref0;     // 100 MHz counter at the start (orders records in time)
  unsigned long long xcc;      // XCC id of the CU that ran the probe
};

__global__ void clock_probe_kernel(ClockRec* rec, unsigned* counter, unsigned cap, unsigned ticks) {
  if (threadIdx.x != 0) return;
  const unsigned i = atomicAdd(counter, 1u);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t1 = t0, r1 = r0;
  while (r1 - r0 < ticks) {
    __builtin_amdgcn_s_sleep(1);
    t1 = __builtin_amdgcn_s_memtime();
    r1 = __builtin_amdgcn_s_memrealtime();
  }
  if (i < cap) {
    ClockRec c;
    c.d_sclk = t1 - t0;
    c.d_ref = r1 - r0;
    c.ref0 = r0;
    c.xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));   // HW_REG_XCC_ID bits [3:0]
    rec[i] = c;
  }
}

LJS_API int ljs_clock_probe(void* rec, void* counter, unsigned cap, unsigned ticks, hipStream_t s) {
  if (ticks < 10 || ticks > 100000) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, s, (ClockRec*)rec, (unsigned*)counter, cap, ticks);
  return (int)hipGetLastError();
}
