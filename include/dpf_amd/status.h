// status.h — absl::Status / absl::StatusOr stand-ins with the same codes and
// accessors (the reference uses Abseil, which is not available here).
#ifndef DPF_AMD_STATUS_H_
#define DPF_AMD_STATUS_H_

#include <optional>
#include <string>
#include <utility>

namespace distributed_point_functions {

// Numbers equal absl::StatusCode.
enum class StatusCode : int {
  kOk = 0,
  kInvalidArgument = 3,
  kResourceExhausted = 8,
  kFailedPrecondition = 9,
  kUnimplemented = 12,
  kInternal = 13,
};

class Status {
 public:
  Status() = default;
  Status(StatusCode code, std::string message)
      : code_(code), message_(std::move(message)) {}
  bool ok() const { return code_ == StatusCode::kOk; }
  StatusCode code() const { return code_; }
  int raw_code() const { return static_cast<int>(code_); }
  const std::string& message() const { return message_; }
  std::string ToString() const;

 private:
  StatusCode code_ = StatusCode::kOk;
  std::string message_;
};

inline Status OkStatus() { return Status(); }
inline Status InvalidArgumentError(std::string m) {
  return Status(StatusCode::kInvalidArgument, std::move(m));
}
inline Status ResourceExhaustedError(std::string m) {
  return Status(StatusCode::kResourceExhausted, std::move(m));
}
inline Status FailedPreconditionError(std::string m) {
  return Status(StatusCode::kFailedPrecondition, std::move(m));
}
inline Status UnimplementedError(std::string m) {
  return Status(StatusCode::kUnimplemented, std::move(m));
}
inline Status InternalError(std::string m) {
  return Status(StatusCode::kInternal, std::move(m));
}

template <typename T>
class StatusOr {
 public:
  StatusOr(const Status& s) : status_(s) {}  // NOLINT
  StatusOr(Status&& s) : status_(std::move(s)) {}  // NOLINT
  StatusOr(const T& v) : value_(v) {}  // NOLINT
  StatusOr(T&& v) : value_(std::move(v)) {}  // NOLINT
  template <typename U,
            typename = std::enable_if_t<std::is_constructible<T, U&&>::value &&
                                        !std::is_same<std::decay_t<U>, Status>::value &&
                                        !std::is_same<std::decay_t<U>, StatusOr>::value>>
  StatusOr(U&& v) : value_(T(std::forward<U>(v))) {}  // NOLINT

  bool ok() const { return status_.ok(); }
  const Status& status() const { return status_; }
  const T& value() const& { return *value_; }
  T& value() & { return *value_; }
  T&& value() && { return std::move(*value_); }
  const T& operator*() const& { return *value_; }
  T& operator*() & { return *value_; }
  T&& operator*() && { return std::move(*value_); }
  const T* operator->() const { return &*value_; }
  T* operator->() { return &*value_; }

 private:
  Status status_;
  std::optional<T> value_;
};

#define DPF_AMD_CONCAT_INNER(a, b) a##b
#define DPF_AMD_CONCAT(a, b) DPF_AMD_CONCAT_INNER(a, b)

#define DPF_RETURN_IF_ERROR(expr)                    \
  do {                                               \
    ::distributed_point_functions::Status _st = (expr); \
    if (!_st.ok()) return _st;                       \
  } while (0)

#define DPF_ASSIGN_OR_RETURN_IMPL(tmp, lhs, expr) \
  auto tmp = (expr);                              \
  if (!tmp.ok()) return tmp.status();             \
  lhs = std::move(*tmp)

#define DPF_ASSIGN_OR_RETURN(lhs, expr) \
  DPF_ASSIGN_OR_RETURN_IMPL(DPF_AMD_CONCAT(_statusor_, __LINE__), lhs, expr)

}  // namespace distributed_point_functions

#endif  // DPF_AMD_STATUS_H_
