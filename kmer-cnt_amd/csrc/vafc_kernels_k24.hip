// vafc_kernels_k24.hip -- instantiates the counting kernels for k = 24, 25, 26, 27.
#include "vafc_scan.h"

hipError_t vc_launch_k24(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<24>(A, grid, grid_long, st);
}
hipError_t vc_setup_k24(int lds) { return setup_k<24>(lds); }

hipError_t vc_launch_k25(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<25>(A, grid, grid_long, st);
}
hipError_t vc_setup_k25(int lds) { return setup_k<25>(lds); }

hipError_t vc_launch_k26(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<26>(A, grid, grid_long, st);
}
hipError_t vc_setup_k26(int lds) { return setup_k<26>(lds); }

hipError_t vc_launch_k27(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<27>(A, grid, grid_long, st);
}
hipError_t vc_setup_k27(int lds) { return setup_k<27>(lds); }

