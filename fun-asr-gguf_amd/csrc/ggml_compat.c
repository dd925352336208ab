/* libggml.so / libggml-base.so of the llama.cpp-compatible library set (include/llama_compat.h): the reference
 * loads both before libllama.so and calls ggml_backend_load_all() once (llama.py:186-203). The engine has no
 * backend registry to fill, so this is its whole content. */
void ggml_backend_load_all(void) {}
