// Syntax stub of the TensorFlow op API subset tf_ops/posecnn_tf_ops.cc uses
// (tests/test_tf_ops_source.py compiles the op source against it with
// -fsyntax-only; TensorFlow itself is not in this image).  Not TensorFlow.
#pragma once
#include <cstddef>
#include <cstdint>
#include <initializer_list>
#include <string>
namespace Eigen {
struct GpuDevice { void* stream() const { return nullptr; } };
}  // namespace Eigen
namespace tensorflow {
typedef int32_t int32;
typedef int64_t int64;
typedef uint8_t uint8;
enum DataType { DT_FLOAT, DT_INT32, DT_UINT8 };
struct Status { bool ok() const { return true; } };
namespace errors {
inline Status InvalidArgument(const char*) { return {}; }
inline Status Internal(const char*) { return {}; }
}  // namespace errors
struct TensorShape {
  TensorShape() {}
  TensorShape(std::initializer_list<int64_t>) {}
};
template <typename T>
struct Flat { T* data() const { return nullptr; } };
struct Tensor {
  int dims() const { return 0; }
  int64_t dim_size(int) const { return 0; }
  int64_t NumElements() const { return 0; }
  TensorShape shape() const { return {}; }
  void* data() const { return nullptr; }
  template <typename T>
  Flat<T> flat() const { return {}; }
};
struct OpKernelConstruction {
  template <typename T>
  Status GetAttr(const char*, T*) { return {}; }
};
struct OpKernelContext {
  const Tensor& input(int) { static Tensor t; return t; }
  Status allocate_output(int, const TensorShape&, Tensor**) { return {}; }
  Status allocate_temp(DataType, const TensorShape&, Tensor*) { return {}; }
  template <typename D>
  const D& eigen_device() { static D d; return d; }
};
struct OpKernel {
  explicit OpKernel(OpKernelConstruction*) {}
  virtual ~OpKernel() {}
  virtual void Compute(OpKernelContext*) = 0;
};
struct OpDefBuilder {
  explicit OpDefBuilder(const char*) {}
  OpDefBuilder& Attr(const char*) { return *this; }
  OpDefBuilder& Input(const char*) { return *this; }
  OpDefBuilder& Output(const char*) { return *this; }
};
struct KernelDefBuilder {
  explicit KernelDefBuilder(const char*) {}
  KernelDefBuilder& Device(const char*) { return *this; }
  template <typename T>
  KernelDefBuilder& TypeConstraint(const char*) { return *this; }
};
inline KernelDefBuilder Name(const char* n) { return KernelDefBuilder(n); }
constexpr const char* DEVICE_GPU = "GPU";
}  // namespace tensorflow
#define PCNN_STUB_CAT2(a, b) a##b
#define PCNN_STUB_CAT(a, b) PCNN_STUB_CAT2(a, b)
#define REGISTER_OP(n) static ::tensorflow::OpDefBuilder PCNN_STUB_CAT(op_, __LINE__) = ::tensorflow::OpDefBuilder(n)
#define REGISTER_KERNEL_BUILDER(b, cls)                                                  \
  static ::tensorflow::KernelDefBuilder PCNN_STUB_CAT(kb_, __LINE__) = b;                \
  static_assert(sizeof(cls) > 0, "")
#define OP_REQUIRES(ctx, cond, st) \
  do {                             \
    if (!(cond)) { (void)(st); return; } \
  } while (0)
#define OP_REQUIRES_OK(ctx, st) \
  do {                          \
    if (!(st).ok()) return;     \
  } while (0)
