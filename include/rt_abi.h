/*
 * rt_abi.h — byte-exact host<->device data ABI of the reference hot path.
 *
 * These are the reference's own drop-in data types, restated as plain C so that
 * the C-ABI (rt_mi355x.h), the HIP kernels and the CPU oracle share one layout:
 *
 *   Sphere          <- src/scene.h:16-22     (80 B, alignof 16)
 *   Scene           <- src/scene.h:24-29     (41 024 B, sphereAmount @ 40 960)
 *   MaterialType    <- src/scene.h:5-9
 *   TextureType     <- src/scene.h:11-14
 *   RenderCallInfo  <- src/render_call_info.h:5-13, mirrored by the std140 UBO at
 *                      shaders/shader.rgen:13-20 (64 B; t[2] is padding)
 *
 * Offsets were verified against the reference with g++ and are
 * pinned by the static asserts at the bottom of this file.
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* src/scene.h:5-9 */
enum rt_material_type { RT_DIFFUSE = 0, RT_METAL = 1, RT_REFRACTIVE = 2 };
/* src/scene.h:11-14 */
enum rt_texture_type { RT_SOLID = 0, RT_CHECKERED = 1 };

/* src/scene.h:24 — the reference's UBO cap. The MI355X build keeps it for the
 * fixed-size Scene struct but accepts unbounded sphere arrays (storage buffers). */
#define RT_MAX_SPHERE_AMOUNT 512u

/* src/scene.h:16-22 (alignas(16) vec4, alignas(4) u32, u32, alignas(16) vec4[2], float) */
typedef struct rt_vec4 { float x, y, z, w; } rt_vec4;

typedef struct __attribute__((aligned(16))) Sphere {
    rt_vec4  geometry;                  /* @0  : center.xyz, radius            */
    uint32_t materialType;              /* @16 : rt_material_type              */
    uint32_t textureType;               /* @20 : rt_texture_type               */
    uint32_t _pad0[2];                  /* @24 : std140 padding                */
    rt_vec4  colors[2];                 /* @32 : solid / checker colours       */
    float    materialSpecificAttribute; /* @64 : metal fuzz or refraction index */
    uint32_t _pad1[3];                  /* @68 : pad to 80                      */
} Sphere;

/* src/scene.h:26-29 (alignas(64) Sphere[512]; alignas(4) u32) */
typedef struct __attribute__((aligned(64))) Scene {
    Sphere   spheres[RT_MAX_SPHERE_AMOUNT];
    uint32_t sphereAmount;
} Scene;

typedef struct rt_uvec2 { uint32_t x, y; } rt_uvec2;

/* src/render_call_info.h:5-13 */
typedef struct __attribute__((aligned(16))) RenderCallInfo {
    uint32_t number;               /* @0  : seed salt (always 0 in the reference, src/ray_trace.cpp:665) */
    uint32_t samplesPerRenderCall; /* @4  : spp of this dispatch (src/ray_trace.cpp:666)                  */
    rt_uvec2 offset;               /* @8  : band offset in the full image (shader.rgen:45)                */
    rt_uvec2 image_size;           /* @16 : full image size (shader.rgen:42)                              */
    uint32_t t[2];                 /* @24 : padding                                                       */
    rt_vec4  camera_pos;           /* @32 : lookFrom (shader.rgen:48)                                     */
    rt_vec4  camera_dir;           /* @48 : lookAt - lookFrom (shader.rgen:49)                            */
} RenderCallInfo;

#ifdef __cplusplus
}  /* extern "C" */
#define RT_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define RT_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif

RT_STATIC_ASSERT(sizeof(Sphere) == 80, "Sphere must be 80 bytes (src/scene.h:16)");
RT_STATIC_ASSERT(offsetof(Sphere, geometry) == 0, "geometry @0");
RT_STATIC_ASSERT(offsetof(Sphere, materialType) == 16, "materialType @16");
RT_STATIC_ASSERT(offsetof(Sphere, textureType) == 20, "textureType @20");
RT_STATIC_ASSERT(offsetof(Sphere, colors) == 32, "colors @32");
RT_STATIC_ASSERT(offsetof(Sphere, materialSpecificAttribute) == 64, "attr @64");
RT_STATIC_ASSERT(sizeof(Scene) == 41024, "Scene must be 41024 bytes");
RT_STATIC_ASSERT(offsetof(Scene, sphereAmount) == 40960, "sphereAmount @40960");
RT_STATIC_ASSERT(sizeof(RenderCallInfo) == 64, "RenderCallInfo must be 64 bytes");
RT_STATIC_ASSERT(offsetof(RenderCallInfo, samplesPerRenderCall) == 4, "spp @4");
RT_STATIC_ASSERT(offsetof(RenderCallInfo, offset) == 8, "offset @8");
RT_STATIC_ASSERT(offsetof(RenderCallInfo, image_size) == 16, "image_size @16");
RT_STATIC_ASSERT(offsetof(RenderCallInfo, camera_pos) == 32, "camera_pos @32");
RT_STATIC_ASSERT(offsetof(RenderCallInfo, camera_dir) == 48, "camera_dir @48");

#endif /* RT_ABI_H */
