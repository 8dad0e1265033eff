// dvh_band_persist.hip -- the band kernel's persistent forms (launch_band_persist: the three-step battery form;
// launch_band_persist_ice: the LP-relaxed ICE form), in a translation unit of their own so that they can be built
// without machine-level loop-invariant code motion (build.py: -mllvm -disable-machine-licm for this file only).  The
// persistent loop runs one window after another in each workgroup; with the hoisting, the window setup's loop
// invariants were kept live across every window's iterations and spilled (dvh_band.hip, launch_band_persist).  The
// kernel itself is dvh_band.hip's.
#define DVH_BAND_PERSIST_TU 1
#include "dvh_band.hip"
