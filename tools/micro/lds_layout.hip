// Prints get_state_kernel's LDS layout constants (simaps.hip) as JSON, for tools/coresidency_model.py.
//   hipcc -std=c++17 -I include -I spatial-intention-maps_amd/csrc tools/micro/lds_layout.hip -o /tmp/lds_layout
#define SIMAPS_DEVICE_ONLY
#include "simaps.hip"
#include <cstdio>
int main()
{
    printf("{\"sizeof_Shared\": %d, \"OFF_DIST\": %d, \"DIST_FLOATS\": %d, \"OFF_UNION\": %d, \"sizeof_SsspScratch\": %d, "
           "\"TILE\": %d, \"TILE_BYTES\": %d, \"CMAP_BYTES\": %d, \"UNION_BYTES\": %d, \"LDS_BYTES\": %d, \"CROP\": %d, \"LW\": %d}\n",
           (int)sizeof(Shared), OFF_DIST, DIST_FLOATS, OFF_UNION, (int)sizeof(SsspScratch), TILE, TILE_BYTES, CMAP_BYTES,
           UNION_BYTES, LDS_BYTES, CROP, LW);
    return 0;
}
