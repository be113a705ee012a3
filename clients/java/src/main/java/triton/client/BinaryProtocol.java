package triton.client;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.charset.StandardCharsets;

import triton.client.pojo.DataType;

/**
 * Little-endian binary tensor encoding of the KServe-v2 binary-data extension
 * (reference BinaryProtocol.java:49-119). Every Java array is written in the
 * width of the declared datatype, so e.g. an int[] may fill an INT8, UINT16 or
 * INT64 tensor; FP16/BF16 are produced from float[]/double[] with
 * round-to-nearest-even.
 */
public final class BinaryProtocol {
  private BinaryProtocol() {}

  private static ByteBuffer alloc(int elems, DataType dt) {
    if (dt.numByte <= 0) throw new IllegalArgumentException(dt + " has no fixed element size");
    return ByteBuffer.allocate(elems * dt.numByte).order(ByteOrder.LITTLE_ENDIAN);
  }

  private static void putIntegral(ByteBuffer b, DataType dt, long v) {
    switch (dt.numByte) {
      case 1: b.put((byte) v); break;
      case 2: b.putShort((short) v); break;
      case 4: b.putInt((int) v); break;
      default: b.putLong(v);
    }
  }

  private static void putFloating(ByteBuffer b, DataType dt, double v) {
    switch (dt) {
      case FP16: b.putShort(floatToHalf((float) v)); break;
      case BF16: b.putShort(floatToBf16((float) v)); break;
      case FP32: b.putFloat((float) v); break;
      case FP64: b.putDouble(v); break;
      default: putIntegral(b, dt, (long) v);
    }
  }

  private static void put(ByteBuffer b, DataType dt, double fv, long iv, boolean isFloat) {
    if (dt.isFloating()) {
      putFloating(b, dt, isFloat ? fv : (double) iv);
    } else if (dt == DataType.BOOL) {
      b.put((byte) ((isFloat ? fv != 0 : iv != 0) ? 1 : 0));
    } else {
      putIntegral(b, dt, isFloat ? (long) fv : iv);
    }
  }

  public static byte[] toBytes(DataType dt, boolean[] data) {
    ByteBuffer b = alloc(data.length, dt);
    for (boolean v : data) put(b, dt, 0, v ? 1 : 0, false);
    return b.array();
  }

  public static byte[] toBytes(DataType dt, byte[] data) {
    if (dt.numByte == 1 && dt != DataType.BOOL) return data.clone();
    ByteBuffer b = alloc(data.length, dt);
    for (byte v : data) put(b, dt, 0, dt.signed ? v : (v & 0xffL), false);
    return b.array();
  }

  public static byte[] toBytes(DataType dt, short[] data) {
    ByteBuffer b = alloc(data.length, dt);
    for (short v : data) put(b, dt, 0, v, false);
    return b.array();
  }

  public static byte[] toBytes(DataType dt, int[] data) {
    ByteBuffer b = alloc(data.length, dt);
    for (int v : data) put(b, dt, 0, v, false);
    return b.array();
  }

  public static byte[] toBytes(DataType dt, long[] data) {
    ByteBuffer b = alloc(data.length, dt);
    for (long v : data) put(b, dt, 0, v, false);
    return b.array();
  }

  public static byte[] toBytes(DataType dt, float[] data) {
    ByteBuffer b = alloc(data.length, dt);
    for (float v : data) put(b, dt, v, 0, true);
    return b.array();
  }

  public static byte[] toBytes(DataType dt, double[] data) {
    ByteBuffer b = alloc(data.length, dt);
    for (double v : data) put(b, dt, v, 0, true);
    return b.array();
  }

  /** BYTES elements: 4-byte little-endian length followed by the UTF-8 bytes. */
  public static byte[] toBytes(DataType dt, String[] data) {
    if (dt != DataType.BYTES) throw new IllegalArgumentException("String data needs BYTES, not " + dt);
    byte[][] enc = new byte[data.length][];
    int total = 0;
    for (int i = 0; i < data.length; i++) {
      enc[i] = data[i].getBytes(StandardCharsets.UTF_8);
      total += 4 + enc[i].length;
    }
    ByteBuffer b = ByteBuffer.allocate(total).order(ByteOrder.LITTLE_ENDIAN);
    for (byte[] e : enc) {
      b.putInt(e.length);
      b.put(e);
    }
    return b.array();
  }

  // ------------------------------------------------------------ half floats
  public static short floatToBf16(float f) {
    int bits = Float.floatToRawIntBits(f);
    if (Float.isNaN(f)) return (short) 0x7fc0;
    int rounding = 0x7fff + ((bits >>> 16) & 1);
    return (short) ((bits + rounding) >>> 16);
  }

  public static float bf16ToFloat(short h) { return Float.intBitsToFloat((h & 0xffff) << 16); }

  public static short floatToHalf(float f) {
    int bits = Float.floatToRawIntBits(f);
    int sign = (bits >>> 16) & 0x8000;
    int exp = (bits >>> 23) & 0xff;
    int mant = bits & 0x7fffff;
    if (exp == 0xff) return (short) (sign | 0x7c00 | (mant != 0 ? 0x200 : 0));
    int e = exp - 127 + 15;
    if (e >= 0x1f) return (short) (sign | 0x7c00);
    if (e <= 0) {
      if (e < -10) return (short) sign;
      mant |= 0x800000;
      int shift = 14 - e;
      int half = mant >>> shift;
      int rem = mant & ((1 << shift) - 1);
      int mid = 1 << (shift - 1);
      if (rem > mid || (rem == mid && (half & 1) != 0)) half++;
      return (short) (sign | half);
    }
    int half = (e << 10) | (mant >>> 13);
    int rem = mant & 0x1fff;
    if (rem > 0x1000 || (rem == 0x1000 && (half & 1) != 0)) half++;
    return (short) (sign | half);
  }

  public static float halfToFloat(short h) {
    int v = h & 0xffff;
    int sign = (v & 0x8000) << 16;
    int exp = (v >>> 10) & 0x1f;
    int mant = v & 0x3ff;
    if (exp == 0) {
      if (mant == 0) return Float.intBitsToFloat(sign);
      float m = mant / 1024.0f * (float) Math.pow(2, -14);
      return sign != 0 ? -m : m;
    }
    if (exp == 0x1f) return Float.intBitsToFloat(sign | 0x7f800000 | (mant << 13));
    return Float.intBitsToFloat(sign | ((exp - 15 + 127) << 23) | (mant << 13));
  }
}
