/*
 * ggml.h — the two ggml symbols the reference's example programs use besides
 * bert.h (examples/main.cpp:9-75, test_batch_encode.cpp:10-80 call
 * ggml_time_init / ggml_time_us; server.cpp:2 includes this header).  libbert.so
 * exports them so those sources compile and link unchanged.  There is no ggml
 * tensor runtime here: the compute path is HIP.
 */
#ifndef EMB_GGML_TIME_H
#define EMB_GGML_TIME_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
__attribute__((visibility("default"))) void ggml_time_init(void);
__attribute__((visibility("default"))) int64_t ggml_time_ms(void);
__attribute__((visibility("default"))) int64_t ggml_time_us(void);
#ifdef __cplusplus
}
#endif
#endif
