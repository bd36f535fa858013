package ax.xz.wireguard.noise.crypto;

import java.lang.foreign.MemorySegment;

import static java.lang.foreign.ValueLayout.JAVA_INT;

/**
 * Drop-in for ax.xz.wireguard.noise.crypto.ChaCha20 (reference ChaCha20.java):
 * same state layout helpers; the keystream (libchacha's chacha_cipher /
 * chacha_block_keystream today, chacha-generic.c:81-108) comes from the device.
 */
public class ChaCha20 {
	static void initializeState(byte[] key, byte[] nonce, MemorySegment state, int counter) {
		initializeState(MemorySegment.ofArray(key), MemorySegment.ofArray(nonce), state, counter);
	}

	static void initializeState(MemorySegment key, MemorySegment nonce, MemorySegment state, int counter) {
		if (state.byteSize() != 64)
			throw new IllegalArgumentException("State size must be 64 bytes (is " + state.byteSize() + ")");
		state.setAtIndex(JAVA_INT, 0, 0x61707865);
		state.setAtIndex(JAVA_INT, 1, 0x3320646e);
		state.setAtIndex(JAVA_INT, 2, 0x79622d32);
		state.setAtIndex(JAVA_INT, 3, 0x6b206574);
		state.asSlice(16, 32).copyFrom(key);
		state.setAtIndex(JAVA_INT, 12, counter);
		state.asSlice(52, 12).copyFrom(nonce);
	}

	/**
	 * Reference ChaCha20.chacha20Block (ChaCha20.java:84-104): word 12 := counter, one keystream
	 * block into output. When both segments are native the reference hands `state` itself to
	 * chacha_block_keystream, whose chacha_block_generic advances word 12 (chacha-generic.c:77);
	 * with a heap segment it works on a native copy and the caller's word 12 stays `counter`.
	 * The same side effect is reproduced here.
	 */
	public static void chacha20Block(MemorySegment state, MemorySegment output, int counter) {
		state.setAtIndex(JAVA_INT, 12, counter);
		var zeros = MemorySegment.ofArray(new byte[64]);
		WgAead.aead(WgAead.WG_MODE_CIPHER, state.asSlice(16, 32), state.getAtIndex(JAVA_INT, 13),
			state.getAtIndex(JAVA_INT, 14), state.getAtIndex(JAVA_INT, 15), counter, zeros, null, output.asSlice(0, 64), 64);
		if (state.isNative() && output.isNative())
			state.setAtIndex(JAVA_INT, 12, counter + 1);
	}

	public static void chacha20(MemorySegment key, MemorySegment nonce, MemorySegment input, MemorySegment output, int counter) {
		if (output.byteSize() < input.byteSize())
			throw new IllegalArgumentException("Output buffer must be at least as large as input buffer");
		WgAead.aead(WgAead.WG_MODE_CIPHER, key, ChaCha20Poly1305.word(nonce, 0), ChaCha20Poly1305.word(nonce, 4),
			ChaCha20Poly1305.word(nonce, 8), counter, input, null, output.asSlice(0, input.byteSize()), input.byteSize());
	}

	public static void chacha20(byte[] key, byte[] nonce, MemorySegment input, MemorySegment output, int counter) {
		chacha20(MemorySegment.ofArray(key), MemorySegment.ofArray(nonce), input, output, counter);
	}
}
