// wavefront.h — host-side interface of the wavefront render pipeline (wavefront.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.h"

namespace myrt {

// Per-frame device queues of the wavefront pipeline (sized for the largest selection
// rendered so far on a replica; grown on demand, never inside a timed loop).
struct WaveBuffers {
    int64_t cap_paths = 0;   // P: path slots (8x8-tiled pixels of the selection)
    int32_t cap_lights = 0;
    int32_t cap_depth = 0;
    void* items[2] = {nullptr, nullptr};   // TraceItem ping-pong queues
    void* hits = nullptr;                  // HitOut per trace slot
    void* shadows = nullptr;               // ShadowItem per shadow slot
    void* contrib = nullptr;               // ShadowContrib per shadow slot
    unsigned char* occluded = nullptr;     // per shadow slot
    void* shade = nullptr;                 // ShadeOut per trace slot
    double* lod = nullptr;                 // [(depth+1)][P][3] direct radiance per level
    double* md = nullptr;                  // [depth][P][3] bounce multiplier per level
    int32_t* term = nullptr;               // [P] terminal level (| kMissFlag)
    unsigned long long* rng = nullptr;     // [P][2] PCG32 state, inc
    double* accum = nullptr;               // [P][3] sample sum
    unsigned* qcount = nullptr;            // 8 XCD-homed work counters per traversal launch
    int64_t bytes = 0;
};

int32_t wave_reserve(WaveBuffers& b, int64_t paths, int32_t lights, int32_t depth);
void wave_release(WaveBuffers& b);

// Enqueue one frame (all samples, all bounce levels) for the selected chunks.
// `counters` receives shadow / secondary ray totals (+ work counters when `count`).
int32_t wave_render(const RenderParams& P, WaveBuffers& b, bool bounce, bool count, hipStream_t stream);

}  // namespace myrt
