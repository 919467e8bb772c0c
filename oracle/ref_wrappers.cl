/* ref_wrappers.cl -- TEST INFRASTRUCTURE ONLY.
 *
 * Harness kernels around the reference's own OpenCL source, which is pulled in
 * by #include from /root/reference/opencl (never copied; see build_ref.py).
 * They exist only so the unmodified reference kernels can be driven through
 * the HIP module API on an MI355X to produce the golden vectors:
 *
 *  - ref_fitter: the reference fitter takes its LDS scratch as __local pointer
 *    arguments (bmfr.cpp:363-365); HIP's module launch has no way to bind
 *    those, so this kernel declares the same three arrays and calls fitter().
 *  - ref_accumulate_noisy_data: runs accumulate_noisy_data() on either the
 *    margin work-items (pass 0) or the owner work-items (pass 1).  Launching
 *    pass 0 then pass 1 gives the race-free semantics of SURVEY.md A.4
 *    (margins read the input colours, bmfr.cl:316-322 vs 478-481).
 */
#include "bmfr.cl"

__attribute__((reqd_work_group_size(256, 1, 1)))
__kernel void ref_fitter(
      __global float* restrict weights,
      __global float* restrict mins_maxs,
#if USE_HALF_PRECISION_IN_TMP_DATA
      __global half* restrict tmp_data,
#else
      __global float* restrict tmp_data,
#endif
      const int frame_number) {
   __local float sum_vec[LOCAL_SIZE];
   __local float u_vec[BLOCK_PIXELS];
#if COMPRESSED_R
   __local float3 r_mat[R_EDGE * (R_EDGE + 1) / 2];
#else
   __local float3 r_mat[R_EDGE * R_EDGE];
#endif
   fitter(sum_vec, u_vec, r_mat, weights, mins_maxs, tmp_data, frame_number);
}

__attribute__((reqd_work_group_size(LOCAL_WIDTH, LOCAL_HEIGHT, 1)))
__kernel void ref_accumulate_noisy_data(
      __global float2* restrict out_prev_frame_pixel,
      __global unsigned char* restrict accept_bools,
      const __global float* restrict current_normals,
      const __global float* restrict previous_normals,
      const __global float* restrict current_positions,
      const __global float* restrict previous_positions,
      __global float* restrict current_noisy,
      const __global float* restrict previous_noisy,
      const __global unsigned char* restrict previous_spp,
      __global unsigned char* restrict current_spp,
#if USE_HALF_PRECISION_IN_TMP_DATA
      __global half* restrict tmp_data,
#else
      __global float* restrict tmp_data,
#endif
      const float16 prev_frame_camera_matrix,
      const float2 pixel_offset,
      const int frame_number,
      const int pass) {
   const int2 gid = {get_global_id(0), get_global_id(1)};
   if (gid.x >= WORKSET_WITH_MARGINS_WIDTH || gid.y >= WORKSET_WITH_MARGINS_HEIGHT)
      return;
   const int2 p = gid - BLOCK_EDGE_HALF + BLOCK_OFFSETS[frame_number % BLOCK_OFFSETS_COUNT];
   const int owner = p.x >= 0 && p.x < IMAGE_WIDTH && p.y >= 0 && p.y < IMAGE_HEIGHT;
   if (owner != pass)
      return;
   accumulate_noisy_data(out_prev_frame_pixel, accept_bools, current_normals,
      previous_normals, current_positions, previous_positions, current_noisy,
      previous_noisy, previous_spp, current_spp, tmp_data,
      prev_frame_camera_matrix, pixel_offset, frame_number);
}
