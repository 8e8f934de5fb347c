// Exclusive scan of package sizes -> byte offsets of each package in the body.
// (kept in its own translation unit: hipCUB/rocPRIM headers are heavy)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "ambc_internal.h"

namespace ambc {

hipError_t scan_sizes(const uint64_t* sizes, uint64_t* off, uint32_t count, void* tmp,
                      size_t* tmp_bytes, hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, *tmp_bytes, sizes, off, (int)count, s);
}

}  // namespace ambc
