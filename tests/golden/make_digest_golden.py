"""Writes tests/golden/blob_writer_digests.json: the only reference-held golden vectors on
the chunk path (per-chunk SHA-256).

Source: /root/reference/tests/blob_writer.rs:11-32 (read as text; the values below are
copied data, not code):
  * TEST_DATA         = 100 000 bytes, byte i = i % 255                      (:12-19)
  * TEST_DIGEST_PLAIN = SHA-256(TEST_DATA), DataChunkBuilder::digest without a
                        crypt config (pbs-datastore/src/data_blob.rs:516-536) (:25-28)
  * TEST_DIGEST_ENC   = CryptConfig::compute_digest(TEST_DATA) = SHA-256(TEST_DATA ||
                        id_key) (pbs-tools/src/crypt_config.rs:79-84) with
                        CryptConfig::new([1u8; 32]) (:20-23), id_key =
                        PBKDF2-HMAC-SHA256([1; 32], b"_id_key", 10 rounds, 32 bytes)
                        (crypt_config.rs:42-51)                              (:29-32)
This script checks them with hashlib (the FIPS 180-4 / RFC 8018 functions the reference
calls through openssl) before writing the fixture.
"""
import hashlib
import json
import os

PLAIN = [83, 154, 96, 195, 167, 204, 38, 142, 204, 224, 130, 201, 24, 71, 2, 188, 130, 155, 177, 6,
         162, 100, 61, 238, 38, 219, 63, 240, 191, 132, 87, 238]
ENC = [50, 162, 191, 93, 255, 132, 9, 14, 127, 23, 92, 39, 246, 102, 245, 204, 130, 104, 4, 106,
       182, 239, 218, 14, 80, 17, 150, 188, 239, 253, 198, 117]


def test_data() -> bytes:
    return bytes(i % 255 for i in range(100_000))


def id_key() -> bytes:
    return hashlib.pbkdf2_hmac("sha256", bytes([1] * 32), b"_id_key", 10, 32)


def main():
    data, key = test_data(), id_key()
    assert hashlib.sha256(data).digest() == bytes(PLAIN)
    assert hashlib.sha256(data + key).digest() == bytes(ENC)
    out = {"source": "reference tests/blob_writer.rs:11-32; pbs-tools/src/crypt_config.rs:42-51,79-84",
           "test_data": "100000 bytes, byte i = i % 255",
           "enc_key": "32 x 0x01", "id_key_pbkdf2": {"salt": "_id_key", "rounds": 10, "hash": "sha256"},
           "id_key": key.hex(), "digest_plain": bytes(PLAIN).hex(), "digest_enc": bytes(ENC).hex()}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "blob_writer_digests.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
