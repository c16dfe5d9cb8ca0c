// mm_n13.hip — the kernels and host drivers of padded size N = 8192
// (log2 N = 13), in their own translation unit (mm_impl.hpp).
#include "mm_impl.hpp"

MM_SIZE_ENTRIES(13)
