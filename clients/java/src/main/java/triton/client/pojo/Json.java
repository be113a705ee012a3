package triton.client.pojo;

import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.Iterator;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;

/**
 * Minimal JSON codec so the client has no third-party dependency (the
 * reference pulls in Jackson for this; src/java/.../Util.java:92-111).
 *
 * Writer: Map, List/array (incl. primitive arrays), String, Number,
 * Boolean, null, {@link Unsigned}. Parser: objects to LinkedHashMap,
 * arrays to ArrayList, integers to Long (Double when fractional or
 * out of range), strings, booleans, null.
 */
public final class Json {
  private Json() {}

  /** A uint64 value written without sign. */
  public static final class Unsigned extends Number {
    private final long bits;

    public Unsigned(long bits) { this.bits = bits; }

    @Override public int intValue() { return (int) bits; }

    @Override public long longValue() { return bits; }

    @Override public float floatValue() { return (float) doubleValue(); }

    @Override public double doubleValue() {
      double d = (double) (bits >>> 1) * 2.0;
      return d + (bits & 1);
    }

    @Override public String toString() { return Long.toUnsignedString(bits); }
  }

  // ---------------------------------------------------------------- writer
  public static String write(Object v) {
    StringBuilder sb = new StringBuilder();
    write(sb, v);
    return sb.toString();
  }

  public static byte[] writeBytes(Object v) { return write(v).getBytes(StandardCharsets.UTF_8); }

  @SuppressWarnings("unchecked")
  private static void write(StringBuilder sb, Object v) {
    if (v == null) {
      sb.append("null");
    } else if (v instanceof String) {
      quote(sb, (String) v);
    } else if (v instanceof Boolean || v instanceof Unsigned) {
      sb.append(v.toString());
    } else if (v instanceof Double || v instanceof Float) {
      double d = ((Number) v).doubleValue();
      if (Double.isNaN(d) || Double.isInfinite(d)) {
        sb.append("null");  // JSON has no NaN/Inf
      } else if (v instanceof Float) {
        sb.append(Float.toString((Float) v));
      } else {
        sb.append(Double.toString(d));
      }
    } else if (v instanceof Number) {
      sb.append(((Number) v).longValue());
    } else if (v instanceof Map) {
      sb.append('{');
      boolean first = true;
      for (Map.Entry<String, Object> e : ((Map<String, Object>) v).entrySet()) {
        if (!first) sb.append(',');
        first = false;
        quote(sb, e.getKey());
        sb.append(':');
        write(sb, e.getValue());
      }
      sb.append('}');
    } else if (v instanceof Iterable) {
      sb.append('[');
      Iterator<Object> it = ((Iterable<Object>) v).iterator();
      boolean first = true;
      while (it.hasNext()) {
        if (!first) sb.append(',');
        first = false;
        write(sb, it.next());
      }
      sb.append(']');
    } else if (v.getClass().isArray()) {
      sb.append('[');
      int n = java.lang.reflect.Array.getLength(v);
      for (int i = 0; i < n; i++) {
        if (i > 0) sb.append(',');
        write(sb, java.lang.reflect.Array.get(v, i));
      }
      sb.append(']');
    } else {
      quote(sb, v.toString());
    }
  }

  private static void quote(StringBuilder sb, String s) {
    sb.append('"');
    for (int i = 0; i < s.length(); i++) {
      char c = s.charAt(i);
      switch (c) {
        case '"': sb.append("\\\""); break;
        case '\\': sb.append("\\\\"); break;
        case '\n': sb.append("\\n"); break;
        case '\r': sb.append("\\r"); break;
        case '\t': sb.append("\\t"); break;
        case '\b': sb.append("\\b"); break;
        case '\f': sb.append("\\f"); break;
        default:
          if (c < 0x20) {
            sb.append(String.format("\\u%04x", (int) c));
          } else {
            sb.append(c);
          }
      }
    }
    sb.append('"');
  }

  // ---------------------------------------------------------------- parser
  public static Object parse(String text) {
    Parser p = new Parser(text);
    p.ws();
    Object v = p.value();
    p.ws();
    if (p.pos != text.length()) throw new IllegalArgumentException("trailing characters at " + p.pos);
    return v;
  }

  @SuppressWarnings("unchecked")
  public static Map<String, Object> parseObject(String text) {
    Object v = parse(text);
    if (!(v instanceof Map)) throw new IllegalArgumentException("expected a JSON object");
    return (Map<String, Object>) v;
  }

  /** Row-major flattening of nested lists (JSON "data" may be nested by shape). */
  @SuppressWarnings("unchecked")
  public static List<Object> flatten(List<Object> in) {
    List<Object> out = new ArrayList<>();
    for (Object o : in) {
      if (o instanceof List) {
        out.addAll(flatten((List<Object>) o));
      } else {
        out.add(o);
      }
    }
    return out;
  }

  private static final class Parser {
    final String s;
    int pos;

    Parser(String s) { this.s = s; }

    void ws() {
      while (pos < s.length() && Character.isWhitespace(s.charAt(pos))) pos++;
    }

    char peek() {
      if (pos >= s.length()) throw new IllegalArgumentException("unexpected end of JSON");
      return s.charAt(pos);
    }

    void expect(char c) {
      if (peek() != c) throw new IllegalArgumentException("expected '" + c + "' at " + pos);
      pos++;
    }

    Object value() {
      char c = peek();
      if (c == '{') return object();
      if (c == '[') return array();
      if (c == '"') return string();
      if (s.startsWith("true", pos)) { pos += 4; return Boolean.TRUE; }
      if (s.startsWith("false", pos)) { pos += 5; return Boolean.FALSE; }
      if (s.startsWith("null", pos)) { pos += 4; return null; }
      return number();
    }

    Map<String, Object> object() {
      Map<String, Object> m = new LinkedHashMap<>();
      expect('{');
      ws();
      if (peek() == '}') { pos++; return m; }
      while (true) {
        ws();
        String k = string();
        ws();
        expect(':');
        ws();
        m.put(k, value());
        ws();
        if (peek() == ',') { pos++; continue; }
        expect('}');
        return m;
      }
    }

    List<Object> array() {
      List<Object> l = new ArrayList<>();
      expect('[');
      ws();
      if (peek() == ']') { pos++; return l; }
      while (true) {
        ws();
        l.add(value());
        ws();
        if (peek() == ',') { pos++; continue; }
        expect(']');
        return l;
      }
    }

    String string() {
      expect('"');
      StringBuilder sb = new StringBuilder();
      while (true) {
        char c = s.charAt(pos++);
        if (c == '"') return sb.toString();
        if (c != '\\') { sb.append(c); continue; }
        char e = s.charAt(pos++);
        switch (e) {
          case 'n': sb.append('\n'); break;
          case 'r': sb.append('\r'); break;
          case 't': sb.append('\t'); break;
          case 'b': sb.append('\b'); break;
          case 'f': sb.append('\f'); break;
          case 'u': sb.append((char) Integer.parseInt(s.substring(pos, pos + 4), 16)); pos += 4; break;
          default: sb.append(e);
        }
      }
    }

    Number number() {
      int start = pos;
      boolean frac = false;
      while (pos < s.length()) {
        char c = s.charAt(pos);
        if ((c >= '0' && c <= '9') || c == '-' || c == '+') {
          pos++;
        } else if (c == '.' || c == 'e' || c == 'E') {
          frac = true;
          pos++;
        } else {
          break;
        }
      }
      String t = s.substring(start, pos);
      if (t.isEmpty()) throw new IllegalArgumentException("bad JSON value at " + start);
      if (!frac) {
        try {
          return Long.parseLong(t);
        } catch (NumberFormatException ex) {
          return new java.math.BigInteger(t).doubleValue();
        }
      }
      return Double.parseDouble(t);
    }
  }
}
