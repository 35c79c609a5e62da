// get_state_mixed_kernel (simaps_get_state_mixed, include/simaps.h): Mapper.get_state (envs.py:2068-2185)
// over agents of several configurations in one launch.  The body is get_state_kernel's
// (get_state_body.inc with GS_MIXED 1): each workgroup takes its configuration from the launch's
// table, and its map slot's and stack's offsets from map_off / out_off.  Built into libsimaps.so
// beside simaps.hip, whose device helpers it includes (SIMAPS_DEVICE_ONLY: no other kernel, no C ABI).
#define SIMAPS_DEVICE_ONLY
#include "simaps.hip"

namespace {
__global__ void __launch_bounds__(NT) get_state_mixed_kernel(
    simaps_mixed::MixedCfgs mx, Geometry geo, const simaps_agent *__restrict__ agents,
    const int32_t *__restrict__ agent_cfg, const simaps_env *__restrict__ envs, const simaps_robot *__restrict__ robots,
    const double *__restrict__ paths, const uint8_t *__restrict__ occupancy, const int64_t *__restrict__ map_off,
    const float *__restrict__ overhead, float *__restrict__ state, const int64_t *__restrict__ out_off, unsigned *fault)
{
    const int k = __builtin_amdgcn_readfirstlane(agent_cfg[blockIdx.x]);
    if ((unsigned)k >= (unsigned)mx.n) {
        // a configuration index past the table: reported, and the workgroup writes nothing (any
        // configuration's C channels at out_off[n] could run past the agent's own stack)
        if (threadIdx.x == 0) post_faults(fault, SIMAPS_FAULT_DESCRIPTOR);
        return;
    }
    const simaps_config cfg = mx.cfg[k];
    const int C = mx.C[k];
    const simaps_debug dbg = {};
#define GS_MIXED 1
#include "get_state_body.inc"
#undef GS_MIXED
}
}  // namespace

namespace simaps_mixed {
void launch_get_state_mixed(const MixedCfgs &mx, const simaps::Geometry &geo, int N, const simaps_agent *agents,
                            const int32_t *agent_cfg, const simaps_env *envs, const simaps_robot *robots,
                            const double *paths, const uint8_t *occupancy, const int64_t *map_off,
                            const float *overhead, float *state, const int64_t *out_off, unsigned *fault,
                            hipStream_t stream)
{
    hipLaunchKernelGGL(get_state_mixed_kernel, dim3(N), dim3(NT), 0, stream, mx, geo, agents, agent_cfg, envs, robots,
                       paths, occupancy, map_off, overhead, state, out_off, fault);
}
}  // namespace simaps_mixed
