/*
 * lgs_io.h -- C-ABI of the host-side f4 components:
 * the Carmen log reader, the map / pose-graph savers and the pose-graph
 * Levenberg-Marquardt optimizer.  Built into liblgs_slam_hip.so (C++ host
 * code over liblgs_hip.so); same conventions as lgs_hip.h (plain pointers,
 * int status, LGS_OK == 0, no exceptions across the ABI).
 *
 *   lgs_carmen_load             IO::Carmen::CarmenLogReader::Load
 *                               C/io/carmen/carmen_reader.cpp:11-530
 *   lgs_pose_graph_optimize_lm  Mapping::PoseGraphOptimizerLM::Optimize
 *                               C/mapping/pose_graph_optimizer_lm.cpp:13-338
 *   lgs_robust_loss             Mapping::Loss{Huber,Cauchy,Fair,GemanMcClure,Welsch,DCS,Squared}
 *                               C/mapping/robust_loss_function.cpp:17-188
 *   lgs_map_draw_image          IO::MapSaver::SaveMapCore's image (DrawMap + DrawTrajectory
 *                               + DrawScan, flipped) C/io/map_saver.cpp:278-463
 *   lgs_map_save                IO::MapSaver::SaveMapCore (PNG + metadata JSON)
 *                               C/io/map_saver.cpp:413-532
 *   lgs_pose_graph_save         IO::MapSaver::SavePoseGraph C/io/map_saver.cpp:56-120
 */
#ifndef LGS_IO_H
#define LGS_IO_H

#include "lgs_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* CarmenLogReader::Load over `text` (NUL-terminated log contents).  Records
 * are written as one flat fp64 stream, record after record:
 *   odometry: 0, timestamp, x, y, theta, vx, vy, vtheta
 *   scan:     1, timestamp, n, odom x y theta, velocity x y theta,
 *             relative sensor pose x y theta, minRange, maxRange, minAngle,
 *             maxAngle, angles[n], ranges[n]
 * and the sensor ids NUL-terminated one after another into ids (*ids_bytes,
 * if not NULL, receives the bytes they need, terminators included).  Returns
 * the number of doubles of the stream (at most cap doubles and ids_cap id
 * bytes are written; call again with larger buffers), or -1 when the reader
 * throws (e.g. a PARAM value stod() rejects -- the reference would
 * terminate). */
long long lgs_carmen_load(const char* text, double* out, long long cap, char* ids, long long ids_cap,
                          long long* ids_bytes, int* num_records);

/* PoseGraph::Edge (H/mapping/pose_graph.hpp:120-170) */
typedef struct {
    int start_node_index, end_node_index;
    lgs_pose2d relative_pose;
    double information[9];          /* row-major 3x3 */
} lgs_pose_graph_edge;

/* PoseGraphOptimizerLM ctor arguments (H/mapping/pose_graph_optimizer_lm.hpp:48-57)
 * and the loss (C/slam_launcher.cpp:603-624) */
#define LGS_LM_SPARSE_CHOLESKY   0
#define LGS_LM_CONJUGATE_GRADIENT 1
#define LGS_LOSS_HUBER 0
#define LGS_LOSS_CAUCHY 1
#define LGS_LOSS_FAIR 2
#define LGS_LOSS_GEMAN_MCCLURE 3
#define LGS_LOSS_WELSCH 4
#define LGS_LOSS_DCS 5
#define LGS_LOSS_SQUARED 6
typedef struct {
    int solver;                     /* LGS_LM_* */
    int num_iterations_max;
    double error_tolerance;
    double lambda;                  /* in: the optimizer's damping factor; out: after the call (a member
                                       of the reference's optimizer, carried to its next Optimize) */
    int loss_kind;                  /* LGS_LOSS_* */
    double loss_scale;
} lgs_pose_graph_lm_params;

/* Optimize(nodes, edges): node_poses updated in place; *iterations and
 * *total_error (ComputeTotalError after the last step) may be NULL. */
int lgs_pose_graph_optimize_lm(lgs_pose_graph_lm_params* params, lgs_pose2d* node_poses, int num_nodes,
                               const lgs_pose_graph_edge* edges, int num_edges, int* iterations,
                               double* total_error);

/* out[2i] = Loss(t[i]), out[2i+1] = Weight(t[i]) of loss `kind` (LGS_LOSS_*) */
int lgs_robust_loss(int kind, double scale, const double* t, int n, double* out);

/* MapSaver::Options (H/io/map_saver.hpp) */
typedef struct {
    int draw_trajectory;
    int trajectory_node_index_min, trajectory_node_index_max;
    int draw_scan;                  /* DrawScan of `scan` at scan_pose */
    lgs_pose2d scan_pose;
    const lgs_scan_host* scan;
    int save_metadata;
} lgs_map_save_options;

/* SaveMapCore's image without writing it: *w x *h RGB bytes (rows top to
 * bottom = the PNG's), into rgb when cap >= w*h*3.  LGS_ERR_INVALID_ARG if
 * the map has no allocated patch (undefined in the reference). */
int lgs_map_draw_image(lgs_ctx* ctx, const lgs_map* map, const lgs_pose2d* node_poses, int num_nodes,
                       const lgs_map_save_options* options, uint8_t* rgb, size_t cap, int* w, int* h);
/* SaveMapCore: <file_name>.png and, with save_metadata, <file_name>.json */
int lgs_map_save(lgs_ctx* ctx, const lgs_map* map, const lgs_pose2d* node_poses, int num_nodes,
                 const lgs_map_save_options* options, const char* file_name);
/* SavePoseGraph: <file_name>.posegraph.json; node k is (node_indices[k],
 * node_poses[k], timestamps[k]) */
int lgs_pose_graph_save(const int* node_indices, const lgs_pose2d* node_poses, const double* timestamps,
                        int num_nodes, const lgs_pose_graph_edge* edges, int num_edges, const char* file_name);

/* The saver's PNG encoder on its own: w x h 8-bit RGB (rows top to bottom),
 * filter 0, zlib-deflated, no interlace -- what boost::gil's png_write_view
 * stores for an rgb8 view (C/io/map_saver.cpp:454-463). */
int lgs_png_write_rgb8(const char* file_name, const uint8_t* rgb, int w, int h);

#ifdef __cplusplus
}
#endif

#endif /* LGS_IO_H */
