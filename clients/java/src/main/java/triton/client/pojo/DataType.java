package triton.client.pojo;

/**
 * KServe-v2 tensor datatypes with their element width in bytes (-1 for
 * variable-length BYTES). Reference: src/java/.../pojo/DataType.java:32-48.
 */
public enum DataType {
  BOOL(1, false),
  UINT8(1, false),
  UINT16(2, false),
  UINT32(4, false),
  UINT64(8, false),
  INT8(1, true),
  INT16(2, true),
  INT32(4, true),
  INT64(8, true),
  FP16(2, true),
  BF16(2, true),
  FP32(4, true),
  FP64(8, true),
  BYTES(-1, false);

  /** Bytes per element; -1 for BYTES. */
  public final int numByte;
  /** Whether the type is signed (the reference spells this field "singed"). */
  public final boolean signed;

  DataType(int numByte, boolean signed) {
    this.numByte = numByte;
    this.signed = signed;
  }

  public boolean isFloating() {
    return this == FP16 || this == BF16 || this == FP32 || this == FP64;
  }
}
