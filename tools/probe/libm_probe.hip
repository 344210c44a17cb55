#include <hip/hip_runtime.h>
#include <math.h>
__global__ void k_add(const double* a, double* b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { double x = a[i]; b[i] = sin(x) ; }
}
__global__ void k_div(const double* a, const double* c, double* b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { b[i] = a[i] / c[i]; }
}
__global__ void k_sqrt(const double* a, double* b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { b[i] = sqrt(a[i]); }
}
__global__ void k_cos(const double* a, double* b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { b[i] = cos(a[i]); }
}
__global__ void k_fmod(const double* a, double* b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { b[i] = fmod(a[i], 6.283185307179586); }
}
__global__ void k_fdiv(const float* a, float* b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { b[i] = a[i] / 50.0f; }
}
extern "C" int run(const char* which, const void* a, const void* c, void* b, int n, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  dim3 g((n + 255) / 256), blk(256);
  if (which[0]=='s' && which[1]=='i') hipLaunchKernelGGL(k_add, g, blk, 0, s, (const double*)a, (double*)b, n);
  else if (which[0]=='d') hipLaunchKernelGGL(k_div, g, blk, 0, s, (const double*)a, (const double*)c, (double*)b, n);
  else if (which[0]=='s' && which[1]=='q') hipLaunchKernelGGL(k_sqrt, g, blk, 0, s, (const double*)a, (double*)b, n);
  else if (which[0]=='c') hipLaunchKernelGGL(k_cos, g, blk, 0, s, (const double*)a, (double*)b, n);
  else if (which[0]=='m') hipLaunchKernelGGL(k_fmod, g, blk, 0, s, (const double*)a, (double*)b, n);
  else if (which[0]=='f') hipLaunchKernelGGL(k_fdiv, g, blk, 0, s, (const float*)a, (float*)b, n);
  return (int)hipGetLastError();
}
