// CU-partitioned HIP streams for the two-stage serving pipeline (synth.PipelinedSynthPath): the
// synthesis of batch i+1 runs on one CU partition while the reverb of batch i runs on the other.
// Serving infrastructure with no reference counterpart (the reference synthesises one batch at a
// time on the CPU, ddsp/models/decoder.py:101-136).
//
// Masks, measured on MI355X (tools/cu_map.hip): HIP deals consecutive CU indices over the 8 XCDs
// (indices 0..63 are 8 CUs of every XCD, 64..255 the other 24 of each), and it ignores masks it
// cannot balance (every 4th / 8th index ran on all 256 CUs); work is split evenly over the
// partition's shader engines, so unbalanced partitions run at the pace of their smallest
// (tools/exp_cumask.py: the reverb took 255 us on 48 or 56 CUs, 137 us on 64-96).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "ddsp_hip.h"

extern "C" {

int ddsp_hip_stream_create_cu_masked(const uint32_t* cu_mask, int mask_words, void** stream) {
  if (!cu_mask || mask_words <= 0 || !stream) return DDSP_HIP_EINVAL;
  bool any = false;
  for (int i = 0; i < mask_words; ++i) any = any || cu_mask[i] != 0;
  if (!any) return DDSP_HIP_EINVAL;
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask_words, cu_mask) != hipSuccess) return DDSP_HIP_ELAUNCH;
  *stream = reinterpret_cast<void*>(s);
  return DDSP_HIP_OK;
}

int ddsp_hip_stream_destroy(void* stream) {
  if (!stream) return DDSP_HIP_EINVAL;
  return hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)) == hipSuccess ? DDSP_HIP_OK : DDSP_HIP_ELAUNCH;
}

}  // extern "C"
