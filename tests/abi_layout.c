/* Prints the layout of the picotls plugin types.  Built twice by tests/test_abi.py: against
 * include/picotls_plugin_abi.h alone, and with the reference's picotls.h force-included first (then the
 * restatement steps aside).  Identical output == the engine's objects are ABI-compatible with picotls. */
#include <stdio.h>
#include "ptls_hip.h"
#define F(T, m) printf(#T "." #m " %zu %zu\n", offsetof(T, m), sizeof(((T *)0)->m))
#define S(T) printf(#T " size %zu\n", sizeof(T))
int main(void)
{
    S(ptls_iovec_t); F(ptls_iovec_t, base); F(ptls_iovec_t, len);
    S(ptls_cipher_context_t); F(ptls_cipher_context_t, algo); F(ptls_cipher_context_t, do_dispose);
    F(ptls_cipher_context_t, do_init); F(ptls_cipher_context_t, do_transform);
    S(ptls_cipher_algorithm_t); F(ptls_cipher_algorithm_t, name); F(ptls_cipher_algorithm_t, key_size);
    F(ptls_cipher_algorithm_t, block_size); F(ptls_cipher_algorithm_t, iv_size); F(ptls_cipher_algorithm_t, context_size);
    F(ptls_cipher_algorithm_t, setup_crypto);
    S(ptls_aead_supplementary_encryption_t); F(ptls_aead_supplementary_encryption_t, ctx);
    F(ptls_aead_supplementary_encryption_t, input); F(ptls_aead_supplementary_encryption_t, output);
    S(ptls_aead_context_t); F(ptls_aead_context_t, algo); F(ptls_aead_context_t, dispose_crypto);
    F(ptls_aead_context_t, do_get_iv); F(ptls_aead_context_t, do_set_iv); F(ptls_aead_context_t, do_encrypt_init);
    F(ptls_aead_context_t, do_encrypt_update); F(ptls_aead_context_t, do_encrypt_final); F(ptls_aead_context_t, do_encrypt);
    F(ptls_aead_context_t, do_encrypt_v); F(ptls_aead_context_t, do_decrypt);
    S(ptls_aead_algorithm_t); F(ptls_aead_algorithm_t, name); F(ptls_aead_algorithm_t, confidentiality_limit);
    F(ptls_aead_algorithm_t, integrity_limit); F(ptls_aead_algorithm_t, ctr_cipher); F(ptls_aead_algorithm_t, ecb_cipher);
    F(ptls_aead_algorithm_t, key_size); F(ptls_aead_algorithm_t, iv_size); F(ptls_aead_algorithm_t, tag_size);
    F(ptls_aead_algorithm_t, tls12); F(ptls_aead_algorithm_t, align_bits); F(ptls_aead_algorithm_t, context_size);
    F(ptls_aead_algorithm_t, setup_crypto);
    {   /* the bit-field cannot be offsetof'd: find the byte that changes when it is set */
        struct st_ptls_aead_algorithm_t a;
        unsigned char *p = (unsigned char *)&a;
        memset(&a, 0, sizeof(a));
        ((struct st_ptls_aead_algorithm_t *)&a)->non_temporal = 1;
        for (size_t i = 0; i < sizeof(a); ++i)
            if (p[i])
                printf("ptls_aead_algorithm_t.non_temporal byte %zu value %u\n", i, p[i]);
    }
    S(ptls_cipher_suite_t); F(ptls_cipher_suite_t, id); F(ptls_cipher_suite_t, aead); F(ptls_cipher_suite_t, hash);
    F(ptls_cipher_suite_t, name);
    S(ptls_hip_record_t);
    return 0;
}
