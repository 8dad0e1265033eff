// dvh_band_persist_ice.hip -- the band kernel's persistent LP-relaxed ICE form (launch_band_persist_ice), in a
// translation unit of its own: built without machine-level loop-invariant code motion like the battery form, but with
// the default scheduler (the AMDGPU register-pressure trackers that speed the battery form up cost this one 4.4 % on
// config 5, profiles/r05zg_sched_options.log).  The kernel itself is dvh_band.hip's.
#define DVH_BAND_PERSIST_TU 2
#include "dvh_band.hip"
