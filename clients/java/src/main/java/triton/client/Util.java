package triton.client;

import java.util.Collection;

/** Small helpers (reference Util.java:33-111). */
public final class Util {
  private Util() {}

  public static boolean isEmpty(String s) { return s == null || s.isEmpty(); }

  public static boolean isEmpty(Collection<?> c) { return c == null || c.isEmpty(); }

  /** Number of elements of a tensor shape (1 for a scalar). */
  public static long elemNumFromShape(long[] shape) {
    long n = 1;
    for (long d : shape) {
      if (d < 0) throw new IllegalArgumentException("negative dimension " + d);
      n *= d;
    }
    return n;
  }

  public static byte[] intToBytes(int a) {
    return new byte[] {(byte) a, (byte) (a >>> 8), (byte) (a >>> 16), (byte) (a >>> 24)};
  }

  public static void checkArgument(boolean cond, String fmt, Object... args) {
    if (!cond) throw new IllegalArgumentException(String.format(fmt, args));
  }
}
