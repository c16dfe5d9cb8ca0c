// mm_n05.hip — the kernels and host drivers of padded size N = 32
// (log2 N = 5), in their own translation unit (mm_impl.hpp).
#include "mm_impl.hpp"

MM_SIZE_ENTRIES(5)
