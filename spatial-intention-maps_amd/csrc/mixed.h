// simaps_get_state_mixed: the launch-wide table of configurations (at most SIMAPS_MAX_MIXED) that
// travels in the kernel arguments, and the launcher of get_state_mixed_kernel.  The kernel lives in
// its own translation unit (simaps_mixed.hip), so that adding it cannot change the code the
// compiler makes of the single-configuration kernels in simaps.hip.
#pragma once
#include <hip/hip_runtime.h>
#include "geom.h"
#include "simaps.h"

namespace simaps_mixed {
struct MixedCfgs {
    simaps_config cfg[SIMAPS_MAX_MIXED];
    int C[SIMAPS_MAX_MIXED];  // simaps_num_channels of each configuration
    int n;                    // configurations in use
};
void launch_get_state_mixed(const MixedCfgs &mx, const simaps::Geometry &geo, int N, const simaps_agent *agents,
                            const int32_t *agent_cfg, const simaps_env *envs, const simaps_robot *robots,
                            const double *paths, const uint8_t *occupancy, const int64_t *map_off,
                            const float *overhead, float *state, const int64_t *out_off, unsigned *fault,
                            hipStream_t stream);
}  // namespace simaps_mixed
