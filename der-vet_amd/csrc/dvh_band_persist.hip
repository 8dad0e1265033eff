// dvh_band_persist.hip -- the band kernel's persistent three-step battery form (launch_band_persist), in a translation
// unit of its own so that it can be built without machine-level loop-invariant code motion and with the AMDGPU
// scheduler's own register-pressure trackers (build.py EXTRA_FLAGS).  The persistent loop runs one window after another
// in each workgroup; with the hoisting, the window setup's loop invariants were kept live across every window's
// iterations and spilled (dvh_band.hip, launch_band_persist).  The trackers: bench 274.7k -> 280.4k windows/s at
// identical iterations; the ICE form, 4.4 % slower with them, has its own unit (dvh_band_persist_ice.hip;
// profiles/r05zg_sched_options.log).  The kernel itself is dvh_band.hip's.
#define DVH_BAND_PERSIST_TU 1
#include "dvh_band.hip"
