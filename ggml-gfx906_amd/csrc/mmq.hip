// mmq.hip — tiled MFMA mat-mat (prefill, ne11 > 8). Placeholder until the MFMA tile lands:
// mmq_supported() == false routes every batch through the mat-vec kernel in column groups.
#include "dispatch.h"
#include "qcommon.h"

namespace mi355x {

bool mmq_supported(int, const MmArgs &) { return false; }

hipError_t mmq_launch(int, const MmArgs &, hipStream_t, Scratch &) { return hipErrorNotSupported; }

}  // namespace mi355x
