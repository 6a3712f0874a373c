/*
 * pitt_seg.h -- C ABI of the MI355X-native RANSAC-plane / support / Euclidean-cluster path.
 *
 * Drop-in boundary for the PCL calls inside the reference's segmentation services
 * (paths relative to the reference root, TheEngineRoom-UniGe/pitt_object_table_segmentation):
 *
 *   pitt_plane_segment / _batch   replaces  seg.segment(*inliers, *coefficients)
 *        src/segmentation_services/plane_segmentation_srv.cpp:52-67   (SACMODEL_PLANE, SAC_RANSAC,
 *        optimize = true; FromNormals falls through to the plain plane model for SACMODEL_PLANE)
 *        src/segmentation_services/supports_segmentation_srv.cpp:89-111 (ransacPlaneSegmentator)
 *   pitt_extract_indices          replaces  ExtractIndices<PointXYZ>::filter (positive / negative)
 *        src/segmentation_services/supports_segmentation_srv.cpp:114-127 (removePlaneInliner)
 *   pitt_find_supports            replaces  the body of findSupports
 *        src/segmentation_services/supports_segmentation_srv.cpp:241-361
 *   pitt_euclidean_clusters       replaces  EuclideanClusterExtraction::extract + KdTree
 *        src/segmentation_services/cluster_segmentation_srv.cpp:54-69
 *   pitt_deep_filter              replaces  the deepFiltering loop
 *        src/segmentation_services/deep_filter_srv.cpp:37-44
 *   pitt_transform_cloud          replaces  pcl::transformPointCloud(cloud, out, Matrix4f)
 *        src/obj_segmentation.cpp:248
 *   pitt_unpack_pointcloud2       replaces  fromROSMsg (PointCloud2 -> PointCloud<PointXYZ>)
 *        src/point_cloud_library/pc_manager.cpp:94-104
 *   pitt_voxel_grid               replaces  VoxelGrid<PointXYZ>::filter (PCManager::downSampling)
 *        src/point_cloud_library/pc_manager.cpp:55-67, src/obj_segmentation.cpp:238
 *   pitt_normal_estimation        replaces  NormalEstimation<PointXYZ, Normal>::compute (estimateNormal)
 *        src/point_cloud_library/pc_manager.cpp:68-78
 *   pitt_sphere_segment           replaces  seg.segment in src/segmentation_services/sphere_segmentation_srv.cpp:57-73
 *   pitt_cylinder_segment         replaces  seg.segment in src/segmentation_services/cylinder_segmentation_srv.cpp:110-126
 *   pitt_cone_segment             replaces  seg.segment in src/segmentation_services/cone_segmentation_srv.cpp:111-127
 *   pitt_axis_height              replaces  the projection + O(n^2) height loop after seg.segment in
 *        src/segmentation_services/cylinder_segmentation_srv.cpp:129-189 and
 *        src/segmentation_services/cone_segmentation_srv.cpp:129-189
 *
 * Conventions: plain pointers and sizes, no C++ types, no exceptions.  Every call returns an
 * int status (PITT_OK, PITT_NO_MODEL, or a negative PITT_E_*).  A context is not thread-safe;
 * one context per thread (the reference's handlers run serially under ros::spin, s3.3).
 * "No model" mirrors PCL's cleared outputs: n_inliers = 0, n_coeff = 0.
 * Core results keep exact PCL semantics; the reference's post-processing quirks (drop index 0,
 * centroid / (n+1)) are applied by the service mirror (pitt_srv.h), never here.
 */
#ifndef PITT_SEG_H
#define PITT_SEG_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3: pitt_sac_params.cov_mode (A6), pitt_cylinder_params / pitt_cone_params.eigen33, pitt_build_flags.
 * 4: pitt_graph_stats removed (the plane pipeline launches directly; HIP graphs measured no gain);
 *    pitt_multi_* (frame-sharded plane batches over several devices from one host process);
 *    pitt_find_supports_aos, pitt_euclidean_clusters_aos (host AoS clouds uploaded as they lie).
 * Callers check pitt_abi_version() == PITT_ABI_VERSION when they load the library: the structs passed
 * by pointer are read in this ABI's layout. */
#define PITT_ABI_VERSION 4
/* Points per scoring tile; frames are scored in tiles of this many points. */
#define PITT_TILE_POINTS 2048

enum {
    PITT_OK = 0,
    PITT_NO_MODEL = 1,        /* not an error: RANSAC found no model (PCL clears outputs) */
    PITT_E_INVALID = -1,      /* bad argument (null pointer, misaligned offset, capacity)  */
    PITT_E_HIP = -2,          /* HIP runtime error                                          */
    PITT_E_NOMEM = -3,        /* device or host allocation failed                           */
    PITT_E_SAMPLER = -4,      /* sampler table exhausted (> slack rejected samples)         */
    PITT_E_NODEVICE = -5      /* no gfx950 device / kernels not loadable                    */
};

/* A3: reduction order of the 4-lane Eigen dot / squaredNorm in the reference's PCL build. */
enum { PITT_REDUCE_SSE2 = 0, PITT_REDUCE_HADD = 1, PITT_REDUCE_SEQ = 2 };
/* A9: Eigen 3.2 `v /= s` multiplies by 1/s (default); Eigen >= 3.3 divides. */
enum { PITT_DIV_EIGEN32 = 0, PITT_DIV_TRUE = 1 };
/* A6: optimizeModelCoefficients' covariance.  EXACT (default, the parity path): PCL's nine float
 * accumulators summed sequentially in inlier order.  FAST: the nine sums in double, each (frame,
 * 2048-point tile) summed by one wave and the tiles reduced in a fixed tree -- the whole chip on the
 * batch instead of one serial chain per frame; coefficients within ~1e-6 of EXACT, not bit-equal. */
enum { PITT_COV_EXACT = 0, PITT_COV_FAST = 1 };

typedef struct pitt_ctx pitt_ctx;

/* Parameters of one SACSegmentation call (sac_segmentation.h members the reference sets). */
typedef struct {
    double   threshold;       /* setDistanceThreshold; compared as fabs(float) < double      */
    int32_t  max_iterations;  /* setMaxIterations; RANSAC evaluates at most max_it+1 models  */
    double   probability;     /* RandomSampleConsensus probability_ (PCL default 0.99)       */
    uint32_t seed;            /* model rng seed; PCL uses 12345 (random_ == false)           */
    int32_t  optimize;        /* setOptimizeCoefficients                                     */
    int32_t  reduce_order;    /* PITT_REDUCE_*                                               */
    int32_t  div_mode;        /* PITT_DIV_*                                                  */
    int32_t  sampler_slack;   /* sampler attempts beyond max_it+1 for rejected samples; at least  *
                               * 1000 are always provided (getSamples' consecutive-draw limit)  */
    int32_t  cov_mode;        /* PITT_COV_* (A6); EXACT unless asked                          */
    int32_t  pad;
} pitt_sac_params;

/* plane_segmentation_srv.cpp:19-21 defaults: th 0.007, 1000 iterations, seed 12345. */
void pitt_sac_params_default(pitt_sac_params* p);

/* Per-frame outcome of a plane segmentation (batch or single). */
typedef struct {
    float    coefficients[4];      /* a, b, c, d (refined when optimize)                 */
    int32_t  n_coeff;              /* 4, or 0 when no model                              */
    int32_t  status;               /* PITT_OK / PITT_NO_MODEL / PITT_E_*                 */
    int64_t  n_inliers;            /* final inlier count                                 */
    int32_t  hypotheses;           /* models PCL's RANSAC evaluates (T)                  */
    int32_t  best_hypothesis;      /* index of the winning model                         */
    int64_t  best_count;           /* inliers of the winning (unrefined) model           */
    int32_t  rejected_samples;     /* isSampleGood rejections before the last hypothesis */
    int32_t  flags;                /* PITT_FLAG_*                                        */
} pitt_plane_result;

enum {
    PITT_FLAG_K_NEAR_INTEGER = 1   /* adaptive k within 1e-12 of an integer: libm-sensitive */
};

/* A batch of frames resident in device memory as structure-of-arrays float planes.
 * Frame f holds counts[f] points at x/y/z[offsets[f] ... offsets[f]+counts[f]).
 * offsets[f] must be a multiple of 4 (16-byte aligned rows) and every frame must stay readable
 * up to offsets[f] + round_up(counts[f], PITT_TILE_POINTS) <= capacity (tail is masked). */
typedef struct {
    const float*   x;
    const float*   y;
    const float*   z;
    const int64_t* offsets;   /* host array [n_frames] */
    const int64_t* counts;    /* host array [n_frames] */
    int32_t        n_frames;
    int64_t        capacity;  /* points readable in each plane */
} pitt_frames;

/* --- context --------------------------------------------------------------------------- */
int  pitt_create(pitt_ctx** out, int hip_device);
void pitt_destroy(pitt_ctx* ctx);
/* Run on a caller-owned hipStream_t (NULL = the context's own stream). */
int  pitt_set_stream(pitt_ctx* ctx, void* hip_stream);
/* Copy bytes between any host / device addresses on the context's stream (synchronous): for FFI
 * callers without HIP bindings reading the device-resident outputs (pitt_*_dev). */
int  pitt_memcpy(pitt_ctx* ctx, void* dst, const void* src, int64_t bytes);
/* The adaptive chunk schedule on this context: batches that ran past the scoring chunks the hint
 * scheduled (a continuation finished them), and the chunks the last batch launched up front
 * ($PITT_ADAPTIVE_CHUNKS=0 always launches every chunk). */
int  pitt_schedule_stats(pitt_ctx* ctx, int64_t* continuations, int32_t* last_chunks);
/* Refined plane batches completed with the binade-run refinement (k_xrefine) on this context, and
 * the frames it handed back to the serial chain ($PITT_XREFINE=0 selects the chain for every frame). */
int  pitt_refine_stats(pitt_ctx* ctx, int64_t* batches, int64_t* fallback_frames);
void* pitt_get_stream(pitt_ctx* ctx);
const char* pitt_last_error(pitt_ctx* ctx);
int  pitt_abi_version(void);
/* Build flags of the loaded library: PITT_BUILD_AB_VARIANTS when it is the A/B build
 * (libpitt_seg_ab.so, `make ab`) that reads kernel-variant knobs ($PITT_LANE_SCORE, ...) from the
 * environment.  The product library returns 0 and ignores those variables. */
enum { PITT_BUILD_AB_VARIANTS = 1 };
int  pitt_build_flags(void);

/* --- plane segmentation ------------------------------------------------------------------ */
/* Single cloud from host memory, PCL layout: stride 16 (PointXYZ: x, y, z, pad) or 12.
 * inliers_out (host, capacity n) receives the ascending inlier indices. */
int pitt_plane_segment(pitt_ctx* ctx, const float* xyz, int64_t n, int32_t stride_bytes,
                       const pitt_sac_params* p, int32_t* inliers_out, int64_t* n_inliers,
                       float coeff_out[4], int32_t* n_coeff);

/* Batch of device-resident frames.  results: host [n_frames].  inliers_dev (optional, device
 * int32 [capacity]): frame f's ascending inliers are written at inliers_dev + offsets[f].
 * Synchronous: returns when results are on the host. */
int pitt_plane_segment_batch(pitt_ctx* ctx, const pitt_frames* frames, const pitt_sac_params* p,
                             pitt_plane_result* results, int32_t* inliers_dev);

/* Asynchronous form: enqueues the batch on the context's stream and returns; `results` is filled by
 * pitt_wait (or by the next call on the context).  One batch in flight per context -- overlap
 * consecutive batches with two contexts on two streams.  With the adaptive chunk schedule a frame
 * that needs more scoring chunks than recent batches of the layout did is finished by pitt_wait
 * (the remaining chunks are enqueued there), so inliers_dev and the results are complete only after
 * pitt_wait (or any later call on the context, pitt_memcpy included): device work the caller orders
 * after this call on the stream must follow pitt_wait. */
int pitt_plane_segment_batch_async(pitt_ctx* ctx, const pitt_frames* frames, const pitt_sac_params* p,
                                   pitt_plane_result* results, int32_t* inliers_dev);
int pitt_wait(pitt_ctx* ctx);

/* --- several devices from one host process (frames shard, one gather) ---------
 * The reference's C++ host (obj_segmentation.cpp:381, ransac_segmentation.cpp) is one process; a
 * pitt_multi holds one context per listed device (a device may be listed twice: two contexts on it).
 * pitt_plane_segment_batch_multi takes a batch in HOST memory (pitt_frames with host planes; frames
 * ascending and non-overlapping), gives device g the contiguous frames [g F / G, (g + 1) F / G), uploads
 * each shard, segments it on its device (one host thread per device) and gathers on the host: results
 * [n_frames] in frame order, and (optional) frame f's ascending inliers at inliers_out + offsets[f]
 * (host int32 [capacity]; entries between a frame's inliers and the next frame are unspecified).
 * Byte-equal to one pitt_plane_segment_batch over all the frames. */
typedef struct pitt_multi pitt_multi;
int  pitt_multi_create(pitt_multi** out, const int32_t* hip_devices, int32_t n_devices);
void pitt_multi_destroy(pitt_multi* m);
int32_t pitt_multi_devices(const pitt_multi* m);
/* Device g's context (owned by m): its device-resident entry points, stream and profiler. */
pitt_ctx* pitt_multi_context(pitt_multi* m, int32_t g);
const char* pitt_multi_last_error(const pitt_multi* m);
int pitt_plane_segment_batch_multi(pitt_multi* m, const pitt_frames* host_frames, const pitt_sac_params* p,
                                   pitt_plane_result* results, int32_t* inliers_out);

/* Debug / parity hooks: per-hypothesis inlier counts of the last batch (host [n_frames*cap]),
 * hypotheses beyond a frame's T are unspecified. */
int pitt_last_hypothesis_counts(pitt_ctx* ctx, int32_t frame, int32_t* counts, int32_t cap);

/* --- ExtractIndices ----------------------------------------------------------------------- */
/* Device SoA in/out.  negative == 0: out = in[indices] (in index order);
 * negative == 1: out = in minus indices, order preserving.  indices ascending, unique. */
int pitt_extract_indices(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                         const int32_t* indices_dev, int64_t n_indices, int32_t negative,
                         float* ox, float* oy, float* oz, int64_t* n_out);

/* --- support segmentation (findSupports) -------------------------------------------------- */
typedef struct {
    float   min_iterative_cloud_percentage;  /* default 0.03  (:30)               */
    float   min_iterative_plane_percentage;  /* default 0.03  (:31)               */
    float   horizontal_variance_threshold;   /* default 0.09  (:33)               */
    float   ransac_distance_threshold;       /* default 0.02f (:35)               */
    int32_t ransac_max_iterations;           /* default 10    (:37)               */
    float   horizontal_axis[3];              /* default 0, 0, -1 (:38)            */
    float   edge_remove_offset[3];           /* default 0.02, 0.02, 0.005 (:39)   */
    int32_t reduce_order;
    int32_t div_mode;
} pitt_support_params;
void pitt_support_params_default(pitt_support_params* p);

typedef struct {
    int32_t      n_points;          /* original cloud size                                  */
    const int32_t* idx_map;         /* Support::inliers: n_points ints (level tags / ranks)  */
    float        coefficients[4];   /* support_coefficient_a..d (refined)                   */
    int64_t      n_support;         /* support_cloud size                                    */
    const float* support_xyz;       /* host, 3*n_support (SoA: x block, y block, z block)    */
    int64_t      n_on_support;      /* on_support_cloud size                                 */
    const float* on_support_xyz;    /* host, 3*n_on_support (SoA)                            */
} pitt_support;

typedef struct {
    int32_t            n_supports;
    const pitt_support* supports;   /* valid until the next call on the context */
    int32_t            iterations;  /* RANSAC rounds run by the loop            */
} pitt_support_list;

/* xyz: host SoA (x[n], y[n], z[n]).  The outputs (idx maps, support and on-support SoA clouds) are
 * in the context's pinned host memory, valid until the next support call on the context. */
int pitt_find_supports(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                       const pitt_support_params* p, pitt_support_list* out);
/* The same from the cloud as it lies in the request (supports_segmentation_srv.cpp:246-247: PCL
 * PointXYZ, stride_bytes 16; or packed xyz, 12): one upload of the caller's bytes, deinterleaved on the
 * device.  The service handlers' path. */
int pitt_find_supports_aos(pitt_ctx* ctx, const float* xyz, int64_t n, int32_t stride_bytes,
                           const pitt_support_params* p, pitt_support_list* out);

/* Device-resident form (the cloud a device preprocessing chain left in HBM: pitt_voxel_grid ->
 * pitt_deep_filter -> pitt_transform_cloud, obj_segmentation.cpp:238-248): x/y/z device SoA; every
 * output stays in the context's device arena (valid until the next call on the context). */
typedef struct {
    int32_t      n_points;          /* original cloud size                                       */
    const int32_t* idx_map;         /* device, n_points ints (Support::inliers)                   */
    float        coefficients[4];   /* host: support_coefficient_a..d (refined)                   */
    int64_t      n_support;
    const float* support_xyz;       /* device SoA planes: x at [0], y at [stride], z at [2 stride] */
    int64_t      n_on_support;
    const float* on_support_xyz;    /* device SoA planes, same stride                              */
    int64_t      stride;            /* plane stride (floats) of support_xyz / on_support_xyz       */
} pitt_support_dev;

typedef struct {
    int32_t                 n_supports;
    const pitt_support_dev* supports;
    int32_t                 iterations;
} pitt_support_list_dev;

int pitt_find_supports_dev(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                           const pitt_support_params* p, pitt_support_list_dev* out);

/* --- Euclidean clusters -------------------------------------------------------------------- */
typedef struct {
    int64_t        size;
    const int32_t* indices;   /* ascending */
    float          sum_xyz[3];/* float sums in index order (the handler derives its centroid) */
} pitt_cluster;

typedef struct {
    int32_t             n_clusters;
    const pitt_cluster* clusters;   /* size-descending (PCL order); valid until next call */
} pitt_cluster_list;

/* xyz: host SoA.  tolerance as ClusterTolerance (double, cast to float by PCL);
 * min_size/max_size as setMin/MaxClusterSize. */
int pitt_euclidean_clusters(pitt_ctx* ctx, const float* x, const float* y, const float* z,
                            int64_t n, double tolerance, int32_t min_size, int32_t max_size,
                            pitt_cluster_list* out);
/* The same from a host AoS cloud (cluster_segmentation_srv.cpp:57-58: PointXYZ, stride_bytes 16; or
 * packed xyz, 12), uploaded as it lies and deinterleaved on the device. */
int pitt_euclidean_clusters_aos(pitt_ctx* ctx, const float* xyz, int64_t n, int32_t stride_bytes,
                                double tolerance, int32_t min_size, int32_t max_size, pitt_cluster_list* out);

/* Device-resident form: x/y/z device SoA; each cluster's members (ascending) stay on the device at
 * indices[offset, offset + size); the sums come back to the host. */
typedef struct {
    int64_t size;
    int64_t offset;
    float   sum_xyz[3];
    float   pad;
} pitt_cluster_dev;

typedef struct {
    int32_t                 n_clusters;
    const pitt_cluster_dev* clusters;   /* size-descending (PCL order); valid until the next call */
    const int32_t*          indices;    /* device */
} pitt_cluster_list_dev;

int pitt_euclidean_clusters_dev(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                double tolerance, int32_t min_size, int32_t max_size, pitt_cluster_list_dev* out);

/* --- the support -> cluster glue on the device (obj_segmentation.cpp:261-312) ------------------ */
/* clusterize's parameters (cluster_segmentation_srv.cpp:32-35, 45-54): tolerance 0.03, min rate 0.01,
 * max rate 0.99, min input size 30 (Q6: read from the tolerance's parameter name -- its default). */
typedef struct {
    double  tolerance;
    double  min_rate;
    double  max_rate;
    int32_t min_input_size;
    int32_t pad;
} pitt_cluster_params;
void pitt_cluster_params_default(pitt_cluster_params* p);

typedef struct {
    int32_t support;      /* the support whose on-support cloud the cluster belongs to */
    int32_t pad;
    int64_t size;
    int64_t offset;       /* members at pitt_scene.indices[offset, offset + size): on-support indices */
    float   sum_xyz[3];   /* float sums in index order (the service's centroid = sum / (size + 1), Q7) */
    float   pad2;
} pitt_object;

typedef struct {
    pitt_support_list_dev supports;
    int32_t               n_objects;   /* clusters of every support, support by support, PCL order */
    const pitt_object*    objects;
    const int32_t*        indices;     /* device */
} pitt_scene;

/* findSupports on the device cloud, then clusterize on every support's on-support cloud (supports with
 * fewer than min_input_size points give no clusters; min / max cluster sizes round(n * rate)), with
 * nothing leaving HBM but sizes, coefficients and sums.  Valid until the next call on the context. */
int pitt_segment_objects_dev(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                             const pitt_support_params* sp, const pitt_cluster_params* cp, pitt_scene* out);

/* --- preprocessing in front of findSupports ------------------------------ */
/* deepFiltering, src/segmentation_services/deep_filter_srv.cpp:27-44: points whose z is NaN are
 * dropped; the rest go to "further" when z > threshold, else to "closer", both in input order.
 * deep_threshold follows getServiceFloatParameter (src/point_cloud_library/srv_manager.h:163-167):
 * a value >= 0 is used, anything else selects the service default 3.0 m (deep_filter_srv.cpp:19);
 * used_threshold (optional) receives the value applied.  Device SoA in; device SoA outputs of
 * capacity n each; either output triple may be NULL (that cloud is only counted). */
int pitt_deep_filter(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                     float deep_threshold, float* closer_x, float* closer_y, float* closer_z,
                     int64_t* n_closer, float* further_x, float* further_y, float* further_z,
                     int64_t* n_further, float* used_threshold);

/* pcl::transformPointCloud(cloud, out, Eigen::Matrix4f) as called at src/obj_segmentation.cpp:248
 * (PCL 1.7 common/impl/transforms.hpp): out.k = m(k,0) x + m(k,1) y + m(k,2) z + m(k,3) in float,
 * left to right, no FMA.  matrix: host, row-major 4x4 (the last row is ignored, as the Affine3f
 * PCL builds from it).  dense = cloud.is_dense: when 0, points with a non-finite coordinate are
 * copied unchanged.  Device SoA in and out (out may not alias in). */
int pitt_transform_cloud(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                         const float matrix[16], int32_t dense, float* out_x, float* out_y, float* out_z);

/* fromROSMsg(PointCloud2 -> PointCloud<PointXYZ>) as called by PCManager::cloudForRosMsg,
 * src/point_cloud_library/pc_manager.cpp:94-104: the XYZ fields of a device-
 * resident little-endian PointCloud2 payload into SoA planes, row-major (point r * width + c at byte
 * r * row_step + c * point_step; x, y, z FLOAT32 at off_x, off_y, off_z).  Offsets, point_step and
 * row_step must be multiples of 4 and data 4-byte aligned; PointXYZ (point_step 16, offsets 0/4/8)
 * takes one 16-byte load per point.  data_bytes is the payload size (msg.data.size()); a layout
 * that would read past it is rejected with PITT_E_INVALID before any device access. */
int pitt_unpack_pointcloud2(pitt_ctx* ctx, const void* data, int64_t data_bytes, int32_t width, int32_t height,
                            int32_t point_step, int64_t row_step, int32_t off_x, int32_t off_y, int32_t off_z,
                            float* x, float* y, float* z);

/* pcl::VoxelGrid<PointXYZ> downsampling as called by PCManager::downSampling,
 * src/point_cloud_library/pc_manager.cpp:55-67 (leaf 0.01 m, :19; called at obj_segmentation.cpp:238).
 * PCL 1.7 applyFilter: one output point per occupied leaf, in ascending leaf index
 * (i + j div_x + k div_x div_y); its value is the float mean of the leaf's finite points (sum, then
 * times 1/n).  Non-finite points never count.  When the grid would overflow int32 PCL warns and
 * returns the input unchanged: then out = in, *n_out = n and *flags |= PITT_VOXEL_OVERFLOW_COPY.
 * order: PITT_VOXEL_ORDER_PCL sums each leaf's points in the order PCL's (unstable) std::sort leaves
 * them -- libstdc++'s introsort permutation, reproduced on the device (assumption A10) -- so the
 * centroids are PCL's bit for bit; PITT_VOXEL_ORDER_STABLE sums them in ascending point order (faster;
 * a centroid may then differ from PCL's in its last bits).
 * Device SoA in; device SoA out of capacity n.  Leaf sizes must be > 0. */
#define PITT_VOXEL_OVERFLOW_COPY 1
#define PITT_VOXEL_ORDER_PCL 0
#define PITT_VOXEL_ORDER_STABLE 1
int pitt_voxel_grid(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                    float leaf_x, float leaf_y, float leaf_z, int32_t order, float* out_x, float* out_y,
                    float* out_z, int64_t* n_out, int32_t* flags);

/* The permutation libstdc++'s std::sort gives (key, val) pairs compared by key only, in place on
 * device arrays (the sort inside pitt_voxel_grid's PCL order; exported for its tests).  depth_limit < 0
 * is the library's 2 floor(log2 n); a smaller one reaches its heapsort fallback. */
int pitt_sort_pairs(pitt_ctx* ctx, uint32_t* key, uint32_t* val, int64_t n, int32_t depth_limit);

/* pcl::NormalEstimation<PointXYZ, Normal> with a search::KdTree and setKSearch(k), as called by
 * PCManager::estimateNormal, src/point_cloud_library/pc_manager.cpp:68-78 (k = 50, :18; called at
 * obj_segmentation.cpp:253 and ransac_segmentation.cpp:233).  Per point: the k nearest finite points
 * (exact; k clamped to the finite count) in ascending float distance (dx*dx + dy*dy) + dz*dz, ties by
 * point index; the float covariance over them in that order, eigen33, curvature |l_min / trace|, the
 * normal flipped towards `viewpoint` (NULL = origin, PCL's default).  A non-finite point or fewer than
 * 3 neighbours gives NaN.  Device SoA in; device outputs of n floats each.  neighbours (n * k int32) and
 * neighbour_count (n) are optional device outputs (the lists in summation order).  k in [1, 64]. */
int pitt_normal_estimation(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                           int32_t k, const float viewpoint[3], float* nx, float* ny, float* nz,
                           float* curvature, int32_t* neighbours, int32_t* neighbour_count);

/* The sphere service's seg.segment (sphere_segmentation_srv.cpp:57-73): SACSegmentationFromNormals with
 * SACMODEL_SPHERE falls through to the plain SampleConsensusModelSphere (normals unused).  RANSAC over
 * 4-point samples (A2 sampler, seed), Eigen 3.2's 4 x 4 determinants in float, the radius limits
 * (-DBL_MAX / DBL_MAX = unset; a model outside them counts 0 inliers), PCL's computeModel loop with
 * w^4; optimize: more than 4 inliers refine the centre and radius by least squares of ||p - c|| - r
 * (PCL: Eigen's float Levenberg-Marquardt -- equal within its tolerance, not bit for bit), then the
 * final selectWithinDistance.  x/y/z device SoA; inliers (device, capacity n) ascending.
 * Returns PITT_OK with a model (coef = centre x, y, z, radius), PITT_NO_MODEL without. */
typedef struct {
    double   threshold;       /* 0.007 (sphere_segmentation_srv.cpp:20) */
    int32_t  max_iterations;  /* 1000 (:23) */
    int32_t  optimize;        /* 1 (:61) */
    double   probability;     /* 0.99 (PCL default) */
    double   radius_min, radius_max;  /* 0.005, 0.5 (:21-22) */
    uint32_t seed;            /* 12345 (PCL's SampleConsensusModel) */
    int32_t  pad;
} pitt_sphere_params;
int pitt_sphere_segment(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                        const pitt_sphere_params* params, int32_t* inliers, int64_t* n_inliers, float coef[4],
                        int32_t* hypotheses);
/* The same on a host PointXYZ cloud (x, y, z, pad: 16-byte stride); inliers in host memory. */
int pitt_sphere_segment_host(pitt_ctx* ctx, const float* xyz16, int64_t n, const pitt_sphere_params* params,
                             int32_t* inliers, int64_t* n_inliers, float coef[4], int32_t* hypotheses);

/* The cylinder service's seg.segment (cylinder_segmentation_srv.cpp:110-126): SampleConsensusModelCylinder
 * with normals (2-point samples; the model from the two normal lines' closest points), the radius limits,
 * the normal-weighted distance |w * angle + (1 - w) * |axis distance - r|| < threshold, PCL's
 * computeModel loop with w^2; optimize: the least-squares refinement of sqrPointToLineDistance - r^2
 * (PCL: Eigen's float Levenberg-Marquardt -- the axis and radius equal within its tolerance, the point
 * on the axis may slide along it), the direction normalised, the final selection.  x/y/z and the
 * normals nx/ny/nz: device SoA of n points; inliers (device, capacity n) ascending; coef[7] = point on
 * the axis, direction, radius.  PITT_OK with a model, PITT_NO_MODEL without. */
typedef struct {
    double   threshold;               /* 0.008 (cylinder_segmentation_srv.cpp:24) */
    int32_t  max_iterations;          /* 1000 (:27) */
    int32_t  optimize;                /* 1 (:114) */
    double   probability;             /* 0.99 */
    double   radius_min, radius_max;  /* 0.005, 0.5 (:25-26) */
    double   normal_distance_weight;  /* 0.001 (:23) */
    uint32_t seed;                    /* 12345 */
    int32_t  eigen33;                 /* getAngle3D's normalized(): 0 = Eigen 3.2 (a zero normal or a point on
                                         the axis gives NaN: never an inlier); 1 = Eigen >= 3.3 (the zero
                                         vector stays zero: the angle is pi/2), as pitt_cone_params */
} pitt_cylinder_params;
int pitt_cylinder_segment(pitt_ctx* ctx, const float* x, const float* y, const float* z, const float* nx,
                          const float* ny, const float* nz, int64_t n, const pitt_cylinder_params* params,
                          int32_t* inliers, int64_t* n_inliers, float coef[7], int32_t* hypotheses);
/* The same on host memory: points as PointXYZ (16-byte stride), normals as (nx, ny, nz) triples. */
int pitt_cylinder_segment_host(pitt_ctx* ctx, const float* xyz16, const float* normals3, int64_t n,
                               const pitt_cylinder_params* params, int32_t* inliers, int64_t* n_inliers,
                               float coef[7], int32_t* hypotheses);

/* The cone service's seg.segment (cone_segmentation_srv.cpp:111-127): SampleConsensusModelCone with normals
 * (3-point samples: the apex where the three tangent planes meet, the axis normal to the plane through the
 * unit apex-to-sample offsets, the opening angle the mean of their acosf to it), the opening-angle limits,
 * isModelValid's eps angle against `axis` (the service sets none: zero), the normal-weighted distance
 * |w * angle(normal, cone normal) + (1 - w) * |axis distance - tan(angle) * height|| < threshold, PCL's
 * computeModel loop with w^3; optimize: the least-squares refinement of OptimizationFunctor's residual
 * sqrPointToLineDistance - (tan(angle) |apex - proj|)^2 (PCL: Eigen's float Levenberg-Marquardt -- equal
 * within its tolerance; fewer than 7 inliers leave the model unchanged, as Eigen's LM refuses m < n), the
 * direction normalised, the final selection.  SACSegmentation's radius limits do not reach SACMODEL_CONE.
 * x/y/z, nx/ny/nz: device SoA of n points; inliers (device, capacity n) ascending; coef[7] = apex,
 * axis direction, opening angle.  PITT_OK with a model, PITT_NO_MODEL without. */
typedef struct {
    double   threshold;               /* 0.0055 (cone_segmentation_srv.cpp:25) */
    int32_t  max_iterations;          /* 1000 (:28) */
    int32_t  optimize;                /* 1 (:115) */
    double   probability;             /* 0.99 */
    double   normal_distance_weight;  /* 0.0006 (:24) */
    double   min_angle, max_angle;    /* radians: 10 and 170 degrees (:30-31, converted at :124) */
    double   eps_angle;               /* 0.4 (:29, set at :125) */
    float    axis[3];                 /* 0, 0, 0: the service sets no axis */
    int32_t  eigen33;                 /* 0: Eigen 3.2's normalized() (0 / 0 = NaN: the eps check against the
                                         zero axis never rejects); 1: Eigen >= 3.3 (a zero vector stays zero:
                                         the angle is pi/2, so eps_angle 0.4 rejects every model) */
    uint32_t seed;                    /* 12345 */
    int32_t  pad;
} pitt_cone_params;
int pitt_cone_segment(pitt_ctx* ctx, const float* x, const float* y, const float* z, const float* nx,
                      const float* ny, const float* nz, int64_t n, const pitt_cone_params* params,
                      int32_t* inliers, int64_t* n_inliers, float coef[7], int32_t* hypotheses);
/* The same on host memory: points as PointXYZ (16-byte stride), normals as (nx, ny, nz) triples. */
int pitt_cone_segment_host(pitt_ctx* ctx, const float* xyz16, const float* normals3, int64_t n,
                           const pitt_cone_params* params, int32_t* inliers, int64_t* n_inliers, float coef[7],
                           int32_t* hypotheses);

/* The post-processing of the cylinder and cone services once PCL has fitted the model
 * (cylinder_segmentation_srv.cpp:129-189, cone_segmentation_srv.cpp:129-189; the helpers :53-79).
 * coef[0..5] (host): the model's axis point (cylinder) or apex (cone) and axis direction.  Every point
 * of the cloud is projected on the axis; *height is the largest float distance
 * sqrt((dx*dx + dy*dy) + dz*dz) between two projected points, (*idx1, *idx2) the first pair (i > j)
 * reaching it in the reference's loop order, and centroid[3] the midpoint of that pair
 * (PITT_AXIS_CYLINDER) or coef[0..2] + 3/4 * height * direction (PITT_AXIS_CONE).  With fewer than two
 * points (no pair) height = -1 and idx = -1, as the reference leaves them; the cylinder centroid is then
 * NaN (the reference reads points[-1]).  The reference runs this only when the model has inliers.
 * x/y/z device SoA of n points; px/py/pz optional device outputs (the projected cloud). */
enum { PITT_AXIS_CYLINDER = 0, PITT_AXIS_CONE = 1 };
int pitt_axis_height(pitt_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                     const float coef[6], int32_t mode, float* px, float* py, float* pz, float* height,
                     int32_t* idx1, int32_t* idx2, float centroid[3]);
/* The same on a host PointXYZ cloud (16-byte stride). */
int pitt_axis_height_host(pitt_ctx* ctx, const float* xyz16, int64_t n, const float coef[6], int32_t mode,
                          float* height, int32_t* idx1, int32_t* idx2, float centroid[3]);

/* --- primitive classification of a frame's clusters --------------------------------------- */
/* The loop of ransac_segmentation.cpp:230-302 (clustersAcquisition) for all of a frame's clusters in
 * one call: per cluster the normals (PCManager::estimateNormal, k = 50), the sphere, cylinder, cone and
 * plane services as their handlers run them (sphere_segmentation_srv.cpp:29-96,
 * cylinder_segmentation_srv.cpp:82-216, cone_segmentation_srv.cpp:83-216, plane_segmentation_srv.cpp:
 * 27-74: the same RANSAC, refinement, selection and axis-height post-processing), the responses'
 * inlier lists without index 0 (PCManager::inlierToVectorMsg, Q1), and the arbitration on their sizes
 * (:265-302).  The clusters move through every stage together: the host synchronises once per stage
 * for the frame (about 30 times), not per cluster and service.  Replaces the per-cluster service calls
 * of clustersAcquisition (:239-258). */
enum { PITT_SHAPE_UNKNOWN = 0, PITT_SHAPE_PLANE = 1, PITT_SHAPE_SPHERE = 2, PITT_SHAPE_CONE = 3,
       PITT_SHAPE_CYLINDER = 4 };  /* TXT_*_SHAPE_TAG, ransac_segmentation.cpp:42-46 */
enum { PITT_SRV_SPHERE = 0, PITT_SRV_CYLINDER = 1, PITT_SRV_CONE = 2, PITT_SRV_PLANE = 3 };
typedef struct {
    int32_t              k;                 /* normal neighbours: 50 (pc_manager.cpp:18), 1..64 */
    float                viewpoint[3];      /* the normals' viewpoint: the origin (PCL default) */
    pitt_sac_params      plane;             /* plane service: pitt_sac_params_default */
    pitt_sphere_params   sphere;            /* the services' defaults (pitt_classify_params_default) */
    pitt_cylinder_params cylinder;
    pitt_cone_params     cone;
    float                cone_over_cylinder; /* DEFAULT_CONE_OVER_CYLINDER_PRIORITY 0.9 (:37) */
    int32_t              pad;
} pitt_classify_params;
void pitt_classify_params_default(pitt_classify_params* p);
typedef struct {
    int64_t n_points;
    int32_t tag;              /* PITT_SHAPE_*: the arbitration */
    int32_t inliers[4];       /* [PITT_SRV_*] the response's inlier count (index 0 dropped, Q1) */
    int32_t status[4];        /* PITT_OK (a model) / PITT_NO_MODEL / error */
    int32_t hypotheses[4];    /* the services' RANSAC iterations */
    int32_t n_coef[4];        /* response coefficients: 4 / 4 with a model (else 0); cylinder and cone
                                 7 + height with a model, else just the height -1 */
    float   sphere[4];        /* centre, radius */
    float   cylinder[8];      /* axis point, direction, radius, height */
    float   cone[8];          /* apex, direction, opening angle, height */
    float   plane[4];
    float   centroid[4][3];   /* the responses' x/y/z_centroid (plane: 0; without inliers: 0) */
    float   est_centroid[3];  /* the chosen primitive's centroid (TrackedShape x/y/z_est_centroid) */
    int32_t pad;
} pitt_cluster_shape;
/* x/y/z: device (or host) SoA; cluster c = points [offsets[c], offsets[c] + counts[c]) (host arrays).
 * out: host [n_clusters]. */
int pitt_classify_clusters(pitt_ctx* ctx, const float* x, const float* y, const float* z, const int64_t* offsets,
                           const int64_t* counts, int32_t n_clusters, const pitt_classify_params* params,
                           pitt_cluster_shape* out);

/* --- synthetic organised clouds (tools; deterministic from scene_seed) ---------------------- */
enum { PITT_SCENE_TABLE = 0, PITT_SCENE_CLUTTER = 1, PITT_SCENE_TABLE_NAN = 2 };
/* 640x480 Kinect-like pinhole cloud in the camera optical frame, row-major pixel order.
 * Writes width*height points into x, y, z. */
int pitt_synth_frame(int32_t scene, uint64_t scene_seed, int32_t width, int32_t height,
                     float* x, float* y, float* z);
/* `views` views of one table scene, transformed to a z-up world frame and concatenated. */
int pitt_synth_fused(uint64_t scene_seed, int32_t views, int32_t width, int32_t height,
                     float* x, float* y, float* z);

/* --- host helpers (no device needed) ------------------------------------------------------- */
/* A2: attempts*3 indices that SampleConsensusModel::drawIndexSample yields for a cloud of n points
 * (mt19937 seeded `seed`, rnd() = mt() >> 1, persistent shuffled index vector). */
int pitt_sampler_table(int64_t n, uint32_t seed, int64_t attempts, int32_t* out);
/* A4: the float t with  (double)fabsf(d) < threshold  <=>  fabsf(d) < t  for every float d. */
float pitt_float_threshold(double threshold);

/* --- profiling ------------------------------------------------------------------------------ */
/* When enabled, every kernel launch is bracketed by hipEvents on the launch stream. */
int pitt_profile_enable(pitt_ctx* ctx, int32_t on);
/* Per-kernel totals since enable: launches, total milliseconds, algorithmic bytes. */
int pitt_profile_get(pitt_ctx* ctx, const char* kernel, int64_t* launches, double* total_ms,
                     double* algorithmic_bytes);
int pitt_profile_reset(pitt_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* PITT_SEG_H */
