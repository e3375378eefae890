"""src/main.py: parse, configure logging, build the codec, run encode/decode, bye()."""
from __future__ import annotations

import logging


def main(parser, CoDec, argv=None):
    args = parser.parse_known_args(argv)[0]
    if args.debug:
        fmt = "(%(levelname)s) %(module)s %(funcName)s %(lineno)d: %(message)s"
        logging.basicConfig(format=fmt, level=logging.DEBUG)
    else:
        logging.basicConfig(format="(%(levelname)s) %(module)s: %(message)s", level=logging.INFO)
    logging.info(f"{args}")
    if getattr(args, "subparser_name", None) is None:
        parser.print_help()
        return 2
    codec = CoDec(args)
    result = args.func(codec)
    codec.bye()
    return result
